"""Bootstrapping latency/throughput on the GPU: Bootstrap
of B level-0 ciphertexts at N = 2^LOGN for each slot count in SLOTS (default
N/2 and N/16); residual chain [60] + [40]x5, bootstrapping chain = residual +
Lattigo v6's default circuit [U]: SlotsToCoeffs 3 (39-bit), EvalMod 8 (60-bit:
the degree-30 CosDiscrete cosine + 3 double angles), CoeffsToSlots 4 (56-bit),
P = [61] x 8 (logPs).  Sparse slot counts run the n-point circuit (trace, one
packed EvalMod) and the post-scale; their inputs have slots >= n zeroed and
their outputs are checked against the replicated n slots.  Prints one JSON
line per (slots, batch) (the first call generates the rotation keys and is
not timed)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.backend import HipLibrary  # noqa: E402


def main():
    logn = int(os.environ.get("LOGN", 16))
    logq = [60] + [40] * 5  # residual; NewBootstrapper extends it
    lib = HipLibrary().new_scheme(logn, logq, [60, 60], 40, h=192, seed=9)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    n = lib.N // 2
    rng = np.random.default_rng(0)
    for ns in [int(eval(x, {"n": n})) for x in os.environ.get("SLOTS", "n,n//16").split(",")]:
        t0 = time.perf_counter()
        lib.NewBootstrapper([61] * 8, ns)
        setup = time.perf_counter() - t0
        for B in [int(b) for b in os.environ.get("BATCH", "1,8").split(",")]:
            vals = rng.uniform(-1, 1, (B, n)).astype(np.float32)
            vals[:, ns:] = 0
            ct = lib.Encrypt(lib.encode_batch(vals, 0, 1 << 40))
            lib.DeleteCiphertext(lib.Bootstrap(ct, ns))  # warm: rotation keys, buffers
            lib.OrionHipSynchronize()
            reps = 3
            t0 = time.perf_counter()
            for _ in range(reps):
                out = lib.Bootstrap(ct, ns)
                lib.OrionHipSynchronize()
                if _ < reps - 1:
                    lib.DeleteCiphertext(out)
            ms = (time.perf_counter() - t0) / reps * 1e3
            dec = lib.decode_f64(lib.Decrypt(out))
            err = np.abs(dec - np.tile(vals[:, :ns], (1, n // ns)).astype(np.float64))
            print(json.dumps({"op": "Bootstrap", "logN": logn, "h": 192, "slots": ns, "batch": B,
                              "ms_per_batch": round(ms, 2), "bootstraps_per_s": round(B / (ms / 1e3), 2),
                              "out_level": lib.GetCiphertextLevel(out),
                              "max_abs_err": float(err.max()), "mean_abs_err": float(err.mean()),
                              "setup_s": round(setup, 2)}), flush=True)
            lib.DeleteCiphertext(out)
            lib.DeleteCiphertext(ct)

if __name__ == "__main__":
    main()
