"""Bootstrap precision probe: error vs N, Hamming weight and message amplitude."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.backend import HipLibrary  # noqa: E402


def run(logn, h, amp, lib):
    logq = [60] + [40] * 5  # residual; NewBootstrapper extends it
    lib.new_scheme(logn, logq, [60, 60], 40, h=h, seed=9)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    n = lib.N // 2
    lib.NewBootstrapper([61], n)
    rng = np.random.default_rng(0)
    vals = (amp * rng.uniform(-1, 1, (1, n))).astype(np.float32)
    ct = lib.Encrypt(lib.encode_batch(vals, 0, 1 << 40))
    d0 = lib.decode_f64(lib.Decrypt(ct))
    out = lib.Bootstrap(ct, n)
    dec = lib.decode_f64(lib.Decrypt(out))
    err = np.abs(dec - d0)
    rel = np.abs(dec - d0).sum() / np.abs(d0).sum()
    print(f"logN={logn} h={h} amp={amp}: max {err.max():.3e} mean {err.mean():.3e} rel {rel:.3e}", flush=True)
    lib.DeleteScheme()


def main():
    lib = HipLibrary()
    for logn, h, amp in [(13, 192, 1.0), (14, 192, 1.0), (15, 192, 1.0), (15, 32, 1.0), (15, 192, 0.1),
                         (16, 192, 1.0), (16, 192, 0.01)]:
        run(logn, h, amp, lib)


if __name__ == "__main__":
    main()
