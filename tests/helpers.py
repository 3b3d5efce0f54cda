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
