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


def bootstrap_keys(lib, ns):
    """The keys of the bootstrapper for `ns` slots (relinearisation, Galois,
    EvkDenseToSparse, EvkSparseToDense): with the input ciphertext, the only
    inputs the CPU oracle shares with the library.  Everything else in the
    circuit -- the prime chain, F, K, the cosine coefficients, the
    CoeffsToSlots / SlotsToCoeffs diagonals and their encoding, the trace
    elements -- the oracle derives itself (oracle.BtpCircuit)."""
    return dict(rlk=lib.bootstrap_export(ns, "rlk"), d2s=lib.bootstrap_export(ns, "d2s"),
                s2d=lib.bootstrap_export(ns, "s2d"),
                gks={int(g): lib.bootstrap_export(ns, "galois", int(g)) for g in lib.bootstrap_export(ns, "galois_keys")})


def bootstrap_oracle(oracle_mod, lib, logn, log_scale, ns, logp):
    """(bootstrapping-chain Oracle, BtpCircuit) derived by the oracle from the
    scheme's moduli and logPs; checks the library's chain is the same."""
    sm = lib.moduli()
    bq, bp = oracle_mod.btp_chain(logn, sm, lib.L, logp)
    lq, lp = lib.bootstrap_moduli(ns)
    assert (lq, lp) == (bq, bp), "the library's bootstrapping chain differs from the oracle's"
    boot = oracle_mod.Oracle(logn, bq + bp, len(bq), len(bp))
    return boot, oracle_mod.BtpCircuit(boot, log_scale, ns)
