"""Composite minimax sign coefficients at `prec` bits (mpmath), the fixture
that pins GenerateMinimaxSignCoeffs (/root/reference/orion/backend/lattigo/
polyeval.go:90-167 -> Lattigo v6 bignum.GenMinimaxCompositePolynomial [U]).

Restated algorithm [U] (Lattigo v6.2.0 is not vendored; this follows its
published construction):
  stage i (degree d_i, interval [-1, -a_i] U [a_i, 1], a_0 = 2^-logalpha):
    p_i = the degree-d_i minimax approximation of sign on that interval set,
          in the Chebyshev basis on [-1, 1]; sign is odd and the interval set
          symmetric, so p_i is odd (Lattigo zeroes the even coefficients) and
          is the odd minimax fit of 1 on [a_i, 1]; E_i = its error;
    p_i <- p_i / (1 + E_i)                   (its image stays inside [-1, 1])
    a_{i+1} = (1 - E_i) / (1 + E_i)          (the image of [a_i, 1])
  orion (polyeval.go:136-143): the last polynomial halved, + 0.5 on T_0.
The minimax polynomial of each stage is unique, so a Remez exchange converged
far below float64 resolution gives Lattigo's coefficients up to its own
stopping threshold; each coefficient is rounded to float64 once (big.Float
.Float64: round to nearest even, as mpmath's float()).

Usage: python tools/gen_minimax.py  ->  tests/golden/minimax_sign.json
"""
import json
import os

import mpmath as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [([15, 15, 27], 128, 6, 12),   # orion.nn.activation._Sign / ReLU defaults (ResNet-20)
         ([7, 15], 128, 4, 12),
         ([31], 128, 3, 12)]


def cheb_odd(c, x):
    """sum_k c_k T_{2k+1}(x) and its derivative."""
    t0, t1 = mp.mpf(1), x
    u0, u1 = mp.mpf(1), 2 * x  # U_0, U_1
    s = ds = mp.mpf(0)
    k = 0
    m = 1
    while k < len(c):
        if m & 1:
            s += c[k] * t1
            ds += c[k] * m * u0  # T_m' = m U_{m-1}
            k += 1
        t0, t1 = t1, 2 * x * t1 - t0
        u0, u1 = u1, 2 * x * u1 - u0
        m += 1
    return s, ds


def remez_odd_one(n, a, tol):
    """Odd minimax fit p = sum_{k<n} c_k T_{2k+1} of 1 on [a, 1]: (c, E)."""
    xs = [(a + 1) / 2 - (1 - a) / 2 * mp.cos(mp.pi * i / n) for i in range(n + 1)]
    grid = [(a + 1) / 2 - (1 - a) / 2 * mp.cos(mp.pi * j / (64 * n)) for j in range(64 * n + 1)]
    done = 0
    for _ in range(60):
        A = mp.matrix(n + 1, n + 1)
        b = mp.matrix(n + 1, 1)
        for i, x in enumerate(xs):
            for k in range(n):
                A[i, k] = mp.chebyt(2 * k + 1, x)
            A[i, n] = (-1) ** i
            b[i] = 1
        sol = mp.lu_solve(A, b)
        c = [sol[k] for k in range(n)]
        E = abs(sol[n])
        # extrema of e = p - 1: the endpoints and the zeros of p' between them
        d = [cheb_odd(c, x)[1] for x in grid]
        ex = [grid[0]]
        for j in range(len(grid) - 1):
            if d[j] == 0 or (d[j] > 0) != (d[j + 1] > 0):
                ex.append(mp.findroot(lambda x: cheb_odd(c, x)[1], (grid[j], grid[j + 1]), solver="anderson"))
        ex.append(grid[-1])
        ev = [cheb_odd(c, x)[0] - 1 for x in ex]
        # keep an alternating set of n + 1 points with the largest errors
        pts = []
        for x, v in zip(ex, ev):
            if pts and (v >= 0) == (pts[-1][1] >= 0):
                if abs(v) > abs(pts[-1][1]):
                    pts[-1] = (x, v)
                continue
            pts.append((x, v))
        while len(pts) > n + 1:
            if abs(pts[0][1]) < abs(pts[-1][1]):
                pts.pop(0)
            else:
                pts.pop()
        emax = max(abs(v) for _, v in pts)
        if len(pts) < n + 1:
            raise RuntimeError("Remez: lost alternation")
        xs = [x for x, _ in pts]
        rel = (emax - E) / emax
        if rel <= tol or emax - E <= mp.ldexp(1, 16) * mp.eps:  # relative, or absolute (values ~1)
            done += 1  # quadratic convergence: two more exchanges after the threshold
            if done == 3:
                return c, emax
    raise RuntimeError("Remez did not converge: n %d a %s rel %s" % (n, mp.nstr(a, 8), mp.nstr(rel, 5)))


def composite(degrees, prec, logalpha):
    with mp.workprec(prec):
        a = mp.ldexp(mp.mpf(1), -logalpha)
        tol = mp.ldexp(mp.mpf(1), -(prec // 2))
        out = []
        for d in degrees:
            n = (d - 1) // 2 + 1
            c, E = remez_odd_one(n, a, tol)
            s = 1 + E
            p = [mp.mpf(0)] * (d + 1)
            for k in range(n):
                p[2 * k + 1] = c[k] / s
            a = (1 - E) / s
            out.append((p, E))
        last = out[-1][0]
        for i in range(len(last)):
            last[i] = last[i] / 2
        last[0] += mp.mpf(0.5)
        return [[float(v) for v in p] for p, _ in out], [float(E) for _, E in out]


def main():
    cases = []
    for degrees, prec, logalpha, logerr in CASES:
        polys, errs = composite(degrees, prec, logalpha)
        cases.append({"degrees": degrees, "prec": prec, "logalpha": logalpha, "logerr": logerr,
                      "stage_errors": errs, "coeffs": polys})
        print(degrees, "stage errors", errs)
    path = os.path.join(ROOT, "tests", "golden", "minimax_sign.json")
    with open(path, "w") as f:
        json.dump({"generator": "tools/gen_minimax.py (mpmath %s, Remez at prec bits)" % mp.__version__,
                   "cases": cases}, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
