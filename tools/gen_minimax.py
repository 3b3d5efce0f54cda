"""Composite minimax sign coefficients at `prec` bits (mpmath), the fixture
that pins GenerateMinimaxSignCoeffs (/root/reference/orion/backend/lattigo/
polyeval.go:90-167 -> Lattigo v6 circuits/ckks/minimax.
GenMinimaxCompositePolynomial and utils/bignum.Remez [U]).

Restated algorithm [U] (Lattigo v6.2.0 is not vendored; this follows its
published construction, the same one orion_amd/csrc/hostmath.cpp restates):
  e = 2^-logerr, alpha = 2^-logalpha, a_0 = alpha;
  stage i (degree d_i): the multi-interval Remez approximation of sign on
    [-1 - e, -a_i + e] U [a_i - e, 1 + e] in the Chebyshev basis T_0 .. T_D
    evaluated at x (D = 2 (1 + (d_i + 1) // 2) - 2: 1 + (d_i + 1) // 2 nodes
    per interval), started on each interval's Chebyshev nodes of the first
    kind, exchanging on the extreme points of the error (interval ends and
    the zeros of p'; same-signed neighbours keep the larger; surplus points
    leave as the smaller end point or the adjacent pair with the smallest
    error sum), stopped once (MaxErr - MinErr) / MinErr <= alpha (at most 50
    iterations); the first d_i + 1 coefficients, the even ones set to zero;
  stage i < last: divided by 1 + MaxErr_i; a_{i+1} = (1 - MaxErr_i) / (1 + MaxErr_i);
  orion (polyeval.go:136-143): the last polynomial halved, + 0.5 on T_0.
Each coefficient is rounded to float64 once (big.Float.Float64: round to
nearest even, as mpmath's float()).

Usage: python tools/gen_minimax.py  ->  tests/golden/minimax_sign.json
"""
import json
import os

import mpmath as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [([15, 15, 27], 128, 6, 12),   # orion.nn.activation._Sign / ReLU defaults (ResNet-20)
         ([15, 15, 27], 128, 6, 8),    # the same with a larger scheme error
         ([7, 15], 128, 4, 12),
         ([31], 128, 3, 12)]


def cheb_full(c, x):
    """sum_j c_j T_j(x) and its derivative (T_j' = j U_{j-1})."""
    t0, t1, u0, u1 = mp.mpf(1), x, mp.mpf(1), 2 * x
    s, ds = c[0], mp.mpf(0)
    for j in range(1, len(c)):
        s += c[j] * t1
        ds += c[j] * j * u0
        t0, t1 = t1, 2 * x * t1 - t0
        u0, u1 = u1, 2 * x * u1 - u0
    return s, ds


def sgn(x):
    return mp.mpf(-1) if x < 0 else (mp.mpf(1) if x > 0 else mp.mpf(0))


def remez_multi(iv, nodes_per, threshold, max_iters=50):
    nn = nodes_per * len(iv)
    D = nn - 2
    xs = []
    for a, b in iv:
        for i in range(nodes_per):
            k = nodes_per - i
            xs.append((a + b) / 2 + (b - a) / 2 * mp.cos(mp.pi * (k - mp.mpf(0.5)) / nodes_per))
    G = 64 * (D + 2)
    grids = [[(a + b) / 2 - (b - a) / 2 * mp.cos(mp.pi * j / G) for j in range(G + 1)] for a, b in iv]
    coeffs = maxerr = minerr = None
    for _ in range(max_iters):
        A = mp.matrix(nn, nn)
        rhs = mp.matrix(nn, 1)
        for i, x in enumerate(xs):
            for j in range(D + 1):
                A[i, j] = mp.chebyt(j, x)
            A[i, D + 1] = -1 if i & 1 else 1
            rhs[i] = sgn(x)
        sol = mp.lu_solve(A, rhs)
        coeffs = [sol[j] for j in range(D + 1)]
        pts = []

        def push(x):
            v = cheb_full(coeffs, x)[0] - sgn(x)
            if pts and (v >= 0) == (pts[-1][1] >= 0):
                if abs(v) > abs(pts[-1][1]):
                    pts[-1] = (x, v)
                return
            pts.append((x, v))

        for g in grids:
            dg = [cheb_full(coeffs, x)[1] for x in g]
            push(g[0])
            for j in range(G):
                if not (dg[j] == 0 or (dg[j] > 0) != (dg[j + 1] > 0)):
                    continue
                if dg[j] == 0 and j == 0:
                    continue
                lo, hi, up = g[j], g[j + 1], dg[j] > 0
                for _b in range(100):
                    m = (lo + hi) / 2
                    if (cheb_full(coeffs, m)[1] > 0) == up:
                        lo = m
                    else:
                        hi = m
                push((lo + hi) / 2)
            push(g[-1])
        E = abs(sol[D + 1])
        vmax = max(abs(v) for _, v in pts)
        if vmax < mp.ldexp(1, -100):  # below the arithmetic's resolution
            maxerr, minerr = max(vmax, E), E
            break
        while len(pts) > nn:
            if len(pts) == nn + 1:
                if abs(pts[0][1]) < abs(pts[-1][1]):
                    pts.pop(0)
                else:
                    pts.pop()
                continue
            m = min(range(len(pts) - 1), key=lambda i: (abs(pts[i][1]) + abs(pts[i + 1][1]), i))
            del pts[m:m + 2]
        if len(pts) < nn:
            raise RuntimeError("Remez lost the alternation")
        maxerr = max(abs(v) for _, v in pts)
        minerr = min(abs(v) for _, v in pts)
        xs = [x for x, _ in pts]
        if (maxerr - minerr) / minerr <= threshold:
            break
    return coeffs, maxerr, minerr


def composite(degrees, prec, logalpha, logerr):
    with mp.workprec(prec):
        alpha, e = mp.ldexp(mp.mpf(1), -logalpha), mp.ldexp(mp.mpf(1), -logerr)
        a = alpha
        polys, errs = [], []
        for i, d in enumerate(degrees):
            if i:
                maxI, minI = 1 + errs[-1], 1 - errs[-1]
                polys[-1] = [v / maxI for v in polys[-1]]
                a = minI / maxI
            c, maxerr, _ = remez_multi([(-1 - e, -a + e), (a - e, 1 + e)], 1 + ((d + 1) >> 1), alpha)
            p = [mp.mpf(0) if j % 2 == 0 else c[j] for j in range(d + 1)]
            polys.append(p)
            errs.append(maxerr)
        last = [v / 2 for v in polys[-1]]
        last[0] += mp.mpf(0.5)
        polys[-1] = last
        return [[float(v) for v in p] for p in polys], [float(E) for E in errs]


def main():
    cases = []
    for degrees, prec, logalpha, logerr in CASES:
        polys, errs = composite(degrees, prec, logalpha, logerr)
        cases.append({"degrees": degrees, "prec": prec, "logalpha": logalpha, "logerr": logerr,
                      "stage_errors": errs, "coeffs": polys})
        print(degrees, logalpha, logerr, "stage errors", errs)
    path = os.path.join(ROOT, "tests", "golden", "minimax_sign.json")
    with open(path, "w") as f:
        json.dump({"generator": "tools/gen_minimax.py (mpmath %s, Remez at prec bits)" % mp.__version__,
                   "cases": cases}, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
