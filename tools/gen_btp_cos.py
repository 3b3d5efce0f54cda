"""Fixture: EvalMod's Chebyshev coefficients in mpmath (test infrastructure).

The bootstrapping circuit's mod-1 polynomial (backend.hip make_circuit ->
hostmath.cpp cos_discrete_cheb; oracle_btp_cos) restates Lattigo v6's default
Mod1Type, CosDiscrete [U]: g(x) = a cos(2 pi (x - 1/4) / 2^r), a =
(2 pi)^(-1/2^r), interpolated at nodes on the integers i in [-(K-1), K-1]
that the ModRaise overflow takes, as Chebyshev coefficients of u = x / K on
[-1, 1]; after r double angles y <- 2 y^2 - a^(2^(i+1)) it is
sin(2 pi x) / (2 pi).  At Lattigo's defaults (K = 16, Mod1Degree = 30,
DoubleAngle = 3; bootstrapper.go:33-38 leaves them at their defaults) the 31
nodes are the 31 integers themselves, one each.  This solves the
interpolation system at 60 significant digits and writes
tests/golden/btp_cos.json; tests/test_oracle.py compares the oracle's 80-bit
values against it.

Usage: python tools/gen_btp_cos.py
"""
import json
import os

import mpmath as mp

K, DEGREE, R, LOGMSG = 16, 30, 3, 8


def coeffs(K, degree, r, dps=60):
    mp.mp.dps = dps
    n = degree + 1
    if n != 2 * K - 1:
        raise ValueError("this fixture covers the one-node-per-integer case (degree + 1 = 2K - 1)")
    a = mp.power(2 * mp.pi, -mp.mpf(1) / 2 ** r)
    xs = [mp.mpf(i) for i in range(-(K - 1), K)]
    A = mp.matrix(n, n)
    b = mp.matrix(n, 1)
    for k, x in enumerate(xs):
        for j in range(n):
            A[k, j] = mp.chebyt(j, x / K)
        b[k] = a * mp.cos(2 * mp.pi * (x - mp.mpf(1) / 4) / 2 ** r)
    return list(mp.lu_solve(A, b))


def main():
    c = coeffs(K, DEGREE, R)
    # the interpolant's error within 2^-LogMessageRatio of each integer (where
    # EvalMod's inputs lie), the edges |i| = K - 1 being the worst
    mp.mp.dps = 60
    a = mp.power(2 * mp.pi, -mp.mpf(1) / 2 ** R)
    dev = mp.ldexp(1, -LOGMSG)
    err, err_small = mp.mpf(0), mp.mpf(0)
    for i in range(-(K - 1), K):
        for s in range(-8, 9):
            x = i + dev * s / 8
            u = x / K
            t = [mp.mpf(1), u]
            for _ in range(DEGREE - 1):
                t.append(2 * u * t[-1] - t[-2])
            p = mp.fsum(cj * tj for cj, tj in zip(c, t))
            e = abs(p - a * mp.cos(2 * mp.pi * (x - mp.mpf(1) / 4) / 2 ** R))
            err = max(err, e)
            if abs(i) <= 8:
                err_small = max(err_small, e)
    out = {"K": K, "degree": DEGREE, "r": R, "dps": 60, "log_message_ratio": LOGMSG,
           "note": "CosDiscrete: (2 pi)^(-1/2^r) cos(2 pi (x - 1/4) / 2^r) interpolated at the integers "
                   "-(K-1)..K-1, Chebyshev coefficients of u = x / K on [-1, 1], lowest degree first "
                   "(tools/gen_btp_cos.py)",
           "max_abs_error_on_grid": mp.nstr(err, 6),
           "max_abs_error_near_integers_up_to_8": mp.nstr(err_small, 6),
           "coeffs": [mp.nstr(x, 40) for x in c]}
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "btp_cos.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, "max error", out["max_abs_error_on_grid"], "|i| <= 8:", out["max_abs_error_near_integers_up_to_8"])


if __name__ == "__main__":
    main()
