"""Fixture: EvalMod's Chebyshev coefficients in mpmath (test infrastructure).

The bootstrapping circuit's mod-1 polynomial (backend.hip make_circuit,
oracle_btp_cos) is the Chebyshev interpolant, at the degree+1 Chebyshev nodes
of [-1, 1], of a cos(2 pi (K u - 1/4) / 2^r) with a = (2 pi)^(-1/2^r): after r
double angles y <- 2 y^2 - a^(2^(i+1)) it is sin(2 pi x) / (2 pi), x = K u.
K, degree and r are Lattigo v6's bootstrapping defaults [U] (K = 16,
Mod1Degree = 30, DoubleAngle = 3; bootstrapper.go:33-38 leaves them at their
defaults).  This computes the same coefficients at 60 significant digits and
writes tests/golden/btp_cos.json; tests/test_oracle.py compares the oracle's
80-bit values against it.

Usage: python tools/gen_btp_cos.py
"""
import json
import os

import mpmath as mp

K, DEGREE, R = 16, 30, 3


def coeffs(K, degree, r, dps=60):
    mp.mp.dps = dps
    m = degree + 1
    a = mp.power(2 * mp.pi, -mp.mpf(1) / 2 ** r)
    fx = [a * mp.cos(2 * mp.pi * (K * mp.cos(mp.pi * (k + mp.mpf(1) / 2) / m) - mp.mpf(1) / 4) / 2 ** r)
          for k in range(m)]
    out = []
    for j in range(m):
        acc = mp.fsum(fx[k] * mp.cos(mp.pi * j * (k + mp.mpf(1) / 2) / m) for k in range(m))
        out.append(acc * (1 if j == 0 else 2) / m)
    return out


def main():
    c = coeffs(K, DEGREE, R)
    # the interpolant reproduces the function at the nodes, and its error on
    # [-1, 1] (sampled) bounds EvalMod's approximation error before the double angles
    mp.mp.dps = 60
    a = mp.power(2 * mp.pi, -mp.mpf(1) / 2 ** R)
    err = mp.mpf(0)
    for i in range(2001):
        u = -1 + mp.mpf(2) * i / 2000
        t = [mp.mpf(1), u]
        for _ in range(DEGREE - 1):
            t.append(2 * u * t[-1] - t[-2])
        p = mp.fsum(cj * tj for cj, tj in zip(c, t))
        f = a * mp.cos(2 * mp.pi * (K * u - mp.mpf(1) / 4) / 2 ** R)
        err = max(err, abs(p - f))
    out = {"K": K, "degree": DEGREE, "r": R, "dps": 60,
           "note": "Chebyshev interpolant of (2 pi)^(-1/2^r) cos(2 pi (K u - 1/4) / 2^r) on [-1, 1], "
                   "coefficients lowest degree first (tools/gen_btp_cos.py)",
           "max_abs_error_on_grid": mp.nstr(err, 6),
           "coeffs": [mp.nstr(x, 40) for x in c]}
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "btp_cos.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, "max error", out["max_abs_error_on_grid"])


if __name__ == "__main__":
    main()
