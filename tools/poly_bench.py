"""Polynomial-evaluation throughput on the GPU: a degree-d
Chebyshev approximation of SiLU on [-1, 1] (orion.nn.SiLU's default degree 31,
activation.py:159-164) evaluated on B ciphertexts of the LoLA N=2^15 chain
(LogQ=[60]+[40]x11, LogP=[60,60]) from the top level.  Prints one JSON line:
ms per batch, images/s, levels consumed, max error vs the cleartext function.
Usage: python tools/poly_bench.py [--degree 31] [--batch 64] [--reps 5]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orion_amd.backend import HipLibrary  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--degree", type=int, default=31)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    logq = [60] + [40] * 11
    lib = HipLibrary().new_scheme(15, logq, [60, 60], 40, h=192, seed=5)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    level = len(logq) - 1
    n = lib.N // 2
    rng = np.random.default_rng(0)
    xs = rng.uniform(-1, 1, (a.batch, n)).astype(np.float32)
    ct = lib.Encrypt(lib.encode_batch(xs, level, 1 << 40))
    nodes = np.polynomial.chebyshev.chebpts1(a.degree + 1)
    silu = nodes / (1 + np.exp(-nodes))
    cf = np.polynomial.chebyshev.Chebyshev.fit(nodes, silu, a.degree).coef.astype(np.float32)
    poly = lib.GenerateChebyshev(list(cf), len(cf))
    out = lib.EvaluatePolynomial(ct, poly, 1 << 40)  # warmup (allocations)
    lib.OrionHipSynchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        lib.DeleteCiphertext(out)
        out = lib.EvaluatePolynomial(ct, poly, 1 << 40)
    lib.OrionHipSynchronize()
    ms = (time.perf_counter() - t0) / a.reps * 1e3
    dec = lib.decode_f64(lib.Decrypt(out))
    x = xs.astype(np.float64)
    err = float(np.abs(dec - np.polynomial.chebyshev.chebval(x, cf.astype(np.float64))).max())
    line = {"op": "EvaluatePolynomial (Chebyshev SiLU)", "degree": a.degree, "batch": a.batch,
            "ms_per_batch": round(ms, 3), "images_per_s": round(a.batch / (ms / 1e3), 1),
            "levels_consumed": level - lib.GetCiphertextLevel(out),
            "out_scale_exact": lib.GetCiphertextScaleF(out) == 2.0 ** 40, "max_abs_err_vs_poly": err,
            "max_abs_err_vs_silu": float(np.abs(dec - x / (1 + np.exp(-x))).max())}
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
