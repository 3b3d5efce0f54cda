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


def bootstrap_inputs(lib, ns):
    """The circuit's shared inputs (keys, diagonals, constants) for the oracle."""
    F, gap, K, r, _deg, _slots, _sy, _top, _lb, _kb, _nt, nlt, _nc = lib.bootstrap_export(ns, "params")
    inp = dict(F=int(F), gap=int(gap), K=int(K), r=int(r), cos=lib.bootstrap_export(ns, "cos"),
               poly_scale=2.0 ** 60, trace=lib.bootstrap_export(ns, "trace"), rlk=lib.bootstrap_export(ns, "rlk"))
    inp["lts"] = []
    for k in range(int(nlt)):
        info = lib.bootstrap_export(ns, "lt_info", k)
        level, n1, nd = (int(v) for v in info[:3])
        inp["lts"].append(dict(level=level, N1=n1, idx=[int(v) for v in info[3:]],
                               pts=[lib.bootstrap_export(ns, "lt_diag", (k << 32) | j) for j in range(nd)]))
    inp["gks"] = {int(g): lib.bootstrap_export(ns, "galois", int(g)) for g in lib.bootstrap_export(ns, "galois_keys")}
    inp["mono_i"] = lib.bootstrap_export(ns, "mono_i") if int(gap) == 1 else None
    return inp
