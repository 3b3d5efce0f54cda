"""Shared helpers for the parity tests (test infrastructure)."""
import numpy as np


def rand_poly(rng, moduli, nlimb_mods, N):
    return np.stack([rng.integers(0, moduli[m], N, dtype=np.uint64) for m in nlimb_mods])


def rand_ct(rng, moduli, level, N, B=1):
    out = np.zeros((B, 2, level + 1, N), dtype=np.uint64)
    for b in range(B):
        for c in range(2):
            for j in range(level + 1):
                out[b, c, j] = rng.integers(0, moduli[j], N, dtype=np.uint64)
    return out


SMALL = dict(logn=13, logq=[55, 40, 40, 40, 40, 40], logp=[60, 60])


class SchemeCache:
    """A GPU scheme shared by the tests of a module, rebuilt whenever another
    test has replaced or deleted the process-global scheme since (the library
    keeps one scheme per process, like Lattigo's scheme.go:32), so the tests
    pass in any order or -k selection."""

    def __init__(self):
        self.val = None

    def get(self, make):
        if self.val is None or not self.val[0].scheme_current():
            self.val = None
            self.val = make()
        return self.val
