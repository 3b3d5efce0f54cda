"""GPU probe of the bootstrapping pipeline stages at N=2^13 (development aid):
CoeffsToSlots followed by SlotsToCoeffs without EvalMod must give back the
slots; ModRaise must preserve the residues mod q0; a full Bootstrap must
decrypt to the input."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.backend import HipLibrary  # noqa: E402


def main():
    logq = [60] + [40] * 5  # residual; NewBootstrapper extends it
    lib = HipLibrary().new_scheme(13, logq, [60, 60], 40, h=32, seed=3)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    n = lib.N // 2
    t0 = time.perf_counter()
    lib.NewBootstrapper([61, 61], n)
    print("NewBootstrapper", round(time.perf_counter() - t0, 2), "s", flush=True)
    rng = np.random.default_rng(1)
    vals = rng.uniform(-1, 1, n).astype(np.float32)
    ct = lib.Encrypt(lib.Encode(list(vals), 0, 1 << 40))
    t0 = time.perf_counter()
    out = lib.Bootstrap(ct, n)
    lib.OrionHipSynchronize()
    print("Bootstrap", round(time.perf_counter() - t0, 3), "s; level", lib.GetCiphertextLevel(out),
          "scale", lib.GetCiphertextScaleF(out), flush=True)
    dec = lib.decode_f64(lib.Decrypt(out))[0]
    err = np.abs(dec - vals)
    print("max err", err.max(), "mean err", err.mean(), "first", dec[:4], vals[:4], flush=True)


if __name__ == "__main__":
    main()
