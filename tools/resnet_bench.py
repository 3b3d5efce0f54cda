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


def main():
    st = OrionStream("resnet20_n13", seed=3)
    t0 = time.perf_counter()
    st.keygen()
    st.compile()
    st.lib.OrionHipSynchronize()
    setup = time.perf_counter() - t0
    img = st.reference_input()
    exp = st.arrays["expected_output"].reshape(-1)
    for B in [int(b) for b in os.environ.get("BATCH", "1,8,32").split(",")]:
        ct = st.encrypt_batch(np.repeat(img, B, axis=0))
        st.lib.DeleteCiphertext(st.forward(ct))  # warm (rotation keys, buffers)
        st.lib.OrionHipSynchronize()
        t0 = time.perf_counter()
        out = st.forward(ct)
        st.lib.OrionHipSynchronize()
        dt = time.perf_counter() - t0
        res = st.decrypt_output(out)
        mae = float(np.abs(res - exp[None]).mean())
        print(json.dumps({"workload": "ResNet-20 CIFAR-10 (reference op stream, N=2^13, 42 bootstraps)",
                          "batch": B, "s_per_batch": round(dt, 3), "images_per_s": round(B / dt, 3),
                          "mae_vs_cleartext": mae, "setup_s": round(setup, 1)}), flush=True)
        st.lib.DeleteCiphertext(out)
        st.lib.DeleteCiphertext(ct)


if __name__ == "__main__":
    main()
