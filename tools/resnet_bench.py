"""GPU: ResNet-20 (CIFAR-10, configs/resnet.yml parameters, N=2^13) encrypted
inference throughput: the reference frontend's op stream replayed for a batch
of B images per handle.  One JSON line per batch size."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.replay import OrionStream  # noqa: E402


def _heartbeat():
    import threading
    t0 = time.time()

    def beat():
        while True:
            time.sleep(50)
            print(f"[resnet_bench] alive {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()


def mark(lib):
    """PROF_MARK=1: an idle gap of 0.6 s before and after the timed forward, so a
    rocprofv3 trace can be cut to the inference (tools/pmc_summary.py --resnet
    takes the kernels between the last two gaps; a torch kernel as the marker
    crashed under rocprofv3's kernel trace)."""
    if os.environ.get("PROF_MARK") == "1":
        lib.OrionHipSynchronize()
        time.sleep(0.6)


def main():
    _heartbeat()
    name = os.environ.get("WORKLOAD", "resnet20_n13")
    st = OrionStream(name, seed=3)
    t0 = time.perf_counter()
    st.keygen()
    print(f"[resnet_bench] keygen {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    st.compile()
    st.lib.OrionHipSynchronize()
    setup = time.perf_counter() - t0
    print(f"[resnet_bench] compile done {setup:.1f} s", file=sys.stderr, flush=True)
    img = st.reference_input()
    exp = st.arrays["expected_output"].reshape(-1)
    for B in [int(b) for b in os.environ.get("BATCH", "1,8,32").split(",")]:
        ct = st.encrypt_batch(np.repeat(img, B, axis=0))
        st.lib.DeleteCiphertext(st.forward(ct))  # warm (rotation keys, buffers)
        st.lib.OrionHipSynchronize()
        mark(st.lib)
        t0 = time.perf_counter()
        out = st.forward(ct)
        st.lib.OrionHipSynchronize()
        dt = time.perf_counter() - t0
        mark(st.lib)
        res = st.decrypt_output(out)
        mae = float(np.abs(res - exp[None]).mean())
        print(json.dumps({"workload": f"ResNet-20 CIFAR-10 (reference op stream {name}, "
                                      f"{st.forward_op_counts().get('Bootstrap', 0)} bootstraps)",
                          "batch": B, "s_per_batch": round(dt, 3), "images_per_s": round(B / dt, 3),
                          "mae_vs_cleartext": mae, "argmax_ok": bool(np.argmax(res[0]) == np.argmax(exp)),
                          "setup_s": round(setup, 1), "pools": st.lib.pool_stats()}), flush=True)
        st.lib.DeleteCiphertext(out)
        if os.environ.get("PROF") == "1":
            # one more forward with HIP events around every launch: per-category
            # kernel ms and algorithmic GB/s (profiling serialises the host a little)
            st.lib.OrionHipProfileReset()
            st.lib.OrionHipProfile(1)
            st.lib.DeleteCiphertext(st.forward(ct))
            st.lib.OrionHipSynchronize()
            st.lib.OrionHipProfile(0)
            br = st.lib.profile_read()
            print(json.dumps({"batch": B, "kernel_ms": {k: round(v["ms"], 2) for k, v in br.items()},
                              "launches": {k: v["launches"] for k, v in br.items()},
                              "algorithmic_gbs": {k: round(v["bytes"] / v["ms"] / 1e6, 1)
                                                  for k, v in br.items() if v["ms"] > 0}}), flush=True)
        st.lib.DeleteCiphertext(ct)


if __name__ == "__main__":
    main()
