"""GenerateMinimaxSignCoeffs (polyeval.go:91-167): composite minimax
approximation of sign on [-1, -2^-logalpha] U [2^-logalpha, 1], host-side
compile-time work, so it runs on the CPU.  Parity with Lattigo v6's
GenMinimaxCompositePolynomial [U] is UNPINNED (not in this image, DESIGN.md
§2): both this backend (hostmath.cpp) and the fixture generator
(tools/gen_minimax.py -> tests/golden/minimax_sign.json, mpmath at `prec`
bits) restate Lattigo's construction -- every interval widened by the scheme
error 2^-logerr, the multi-interval Remez stopped at Lattigo's threshold
(MaxErr - MinErr) / MinErr <= 2^-logalpha, each stage but the last divided by
1 + MaxErr -- so the first test pins the arithmetic of that restatement (the
doubles must be equal), not Lattigo-equality.  The other checks
are the contract the caller (orion/nn/activation.py:201-260, _Sign / ReLU)
relies on -- one Chebyshev coefficient vector per degree, intermediate stages
inside [-1, 1], the last stage mapped to [0, 1] -- and the approximation
quality of the composite."""
import json
import os

import numpy as np
import pytest

from orion_amd.backend import HipLibrary


@pytest.fixture(scope="module")
def lib():
    return HipLibrary()


GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "minimax_sign.json")


@pytest.mark.parametrize("case", range(4))
def test_minimax_sign_matches_prec_bit_fixture(lib, case):
    c = json.load(open(GOLDEN))["cases"][case]
    got = np.array(lib.GenerateMinimaxSignCoeffs(c["degrees"], c["prec"], c["logalpha"], c["logerr"], 0))
    exp = np.concatenate([np.array(p, dtype=np.float64) for p in c["coeffs"]])
    assert got.shape == exp.shape
    assert np.array_equal(got, exp), (np.abs(got - exp).max(), int(np.sum(got != exp)))


def _composite(polys, x):
    y = x
    for p in polys:
        y = np.polynomial.chebyshev.chebval(y, p)
    return y


@pytest.mark.parametrize("degrees,logalpha", [([15, 15, 27], 6), ([7, 15], 4), ([31], 3)])
def test_minimax_sign_composite(lib, degrees, logalpha):
    flat = np.array(lib.GenerateMinimaxSignCoeffs(degrees, 128, logalpha, 12, 0))
    assert len(flat) == sum(d + 1 for d in degrees)
    polys = np.split(flat, np.cumsum([d + 1 for d in degrees])[:-1])
    for p in polys[:-1]:
        assert np.all(p[0::2] == 0)  # odd stages
    alpha = 2.0 ** -logalpha
    x = np.concatenate([np.linspace(alpha, 1, 20001), -np.linspace(alpha, 1, 20001)])
    y = x
    for p in polys[:-1]:
        y = np.polynomial.chebyshev.chebval(y, p)
        assert np.abs(y).max() <= 1 + 1e-9  # each stage stays inside the next one's domain
    out = np.polynomial.chebyshev.chebval(y, polys[-1])  # in [0, 1]: (sign + 1) / 2
    err = np.abs(out - (x > 0)).max()
    bound = {(15, 15, 27): 1e-6, (7, 15): 2e-3, (31,): 1e-2}[tuple(degrees)]  # measured 2.7e-7, 8.8e-4, 3.8e-3
    assert err < bound, err


def test_minimax_default_relu_precision(lib):
    """orion's ReLU default (degrees [15, 15, 27], logalpha 6): the composite
    sign error on |x| >= 2^-6 is far below 2^-12 after the third stage."""
    degrees = [15, 15, 27]
    flat = np.array(lib.GenerateMinimaxSignCoeffs(degrees, 128, 6, 12, 0))
    polys = np.split(flat, np.cumsum([d + 1 for d in degrees])[:-1])
    x = np.concatenate([np.linspace(2.0 ** -6, 1, 50001), -np.linspace(2.0 ** -6, 1, 50001)])
    sign = 2 * _composite(polys, x) - 1
    assert np.abs(sign - np.sign(x)).max() < 2.0 ** -12
    # cached: the same call returns the same coefficients
    assert np.array_equal(np.array(lib.GenerateMinimaxSignCoeffs(degrees, 128, 6, 12, 0)), flat)


def test_minimax_sign_depends_on_logerr(lib):
    """logerr (orion's _Sign default 12, activation.py:207-231) widens every
    fit interval by 2^-logerr, as Lattigo's GenMinimaxCompositePolynomial
    does: the coefficients change with it, and the composite still maps
    inputs perturbed by up to 2^-logerr to the right side."""
    degrees = [15, 15, 27]
    a = np.array(lib.GenerateMinimaxSignCoeffs(degrees, 128, 6, 12, 0))
    b = np.array(lib.GenerateMinimaxSignCoeffs(degrees, 128, 6, 8, 0))
    assert a.shape == b.shape and not np.array_equal(a, b)
    polys = np.split(b, np.cumsum([d + 1 for d in degrees])[:-1])
    e = 2.0 ** -8
    x = np.concatenate([np.linspace(2.0 ** -6 - e, 1 + e, 20001), -np.linspace(2.0 ** -6 - e, 1 + e, 20001)])
    out = _composite(polys, x)
    assert np.abs(out - (x > 0)).max() < 1e-4
