"""GenerateMinimaxSignCoeffs (polyeval.go:91-167): composite minimax
approximation of sign on [-1, -2^-logalpha] U [2^-logalpha, 1], host-side
compile-time work, so it runs on the CPU.  Parity with Lattigo v6's
GenMinimaxCompositePolynomial [U] is UNPINNED (not in this image; logerr is
ignored here): the fixture (tools/gen_minimax.py ->
tests/golden/minimax_sign.json) is this backend's own construction computed
again in mpmath at `prec` bits, so the first test pins the arithmetic (the
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


@pytest.mark.parametrize("case", range(3))
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
