"""CPU replay of an Orion op stream on the parity oracle (TEST INFRASTRUCTURE).

Used only by tests/ and by bench.py's cpu_baseline leg.  Mirrors
orion_amd/replay.py, but every operator runs in the single-threaded C
restatement (oracle/ckks_oracle.c) -- the same algorithm the reference's
Lattigo backend runs single-threaded per op (SURVEY.md §8a "where time goes").
Keys come from the oracle's own seeded test keygen.
"""
import os
import sys

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)

from oracle.oracle import Oracle, gen_moduli  # noqa: E402


def _load(name):
    import json
    g = os.path.join(_ROOT, "tests", "golden")
    with open(os.path.join(g, f"{name}_trace.json")) as f:
        trace = json.load(f)
    arrays = dict(np.load(os.path.join(g, f"{name}_arrays.npz"), allow_pickle=False))
    return trace, arrays


class CpuStream:
    def __init__(self, name, seed=99):
        self.trace, self.arrays = _load(name)
        self.meta = self.trace["meta"]
        cfg = self.meta["config"]
        # ConjugateInvariant ring (scheme.go:49-52): degree N, NthRoot 4N (primes = 1 mod 4N), N real slots
        self.ci = cfg.get("ringtype", "standard").lower() == "conjugateinvariant"
        self.logN = cfg["logn"]
        self.L, self.K = len(cfg["logq"]), len(cfg["logp"])
        self.orc = Oracle(self.logN, gen_moduli(self.logN + self.ci, cfg["logq"], cfg["logp"]), self.L, self.K,
                          ci=self.ci)
        self.N = self.orc.N
        self.slots = self.orc.slots
        self.mods = self.orc.moduli
        self.seed = seed
        self.h = cfg["h"]
        self.gks = {}
        self.pts = {}
        self.lts = {}

    # ---- keys ----
    def keygen(self):
        o = self.orc
        self.sk = o.gen_secret(self.seed, self.h)
        s2 = o.mul_coeffs(self.sk, self.sk, list(range(self.L + self.K)))
        self.rlk = o.gen_evk(self.seed + 1, s2, self.sk)

    def galois_key(self, g):
        if g not in self.gks:
            M = (4 if self.ci else 2) * self.N  # NthRoot
            ginv = pow(g, -1, M)
            s_out = self.orc.automorphism_ntt(self.sk, ginv)
            self.gks[g] = self.orc.gen_evk(self.seed + 7 + len(self.gks), self.sk, s_out)
        return self.gks[g]

    # ---- compile ----
    def compile(self):
        o = self.orc
        for ev in self.trace["events"]:
            if ev["phase"] != "compile":
                continue
            if ev["op"] == "Encode":
                vals = self.arrays[ev["arrays"] + "_values"].astype(np.float64)
                lvl, scale = ev["args"][1], ev["args"][2]
                self.pts[ev["ret"]] = (o.encode(vals, float(scale), list(range(lvl + 1))), lvl, float(scale))
            elif ev["op"] == "GenerateLinearTransform":
                idx, _, level, ratio, _ = ev["args"]
                diags = self.arrays[ev["arrays"] + "_diags"].astype(np.float64)
                import math
                N1 = o.find_best_bsgs_n1(idx, int(math.log(ratio)))
                pts = []
                for i, d in enumerate(idx):
                    rot = d & (self.slots - 1)
                    giant = ((rot // N1) * N1) & (self.slots - 1)
                    vec = np.roll(diags[i], giant)  # right rotation by the giant step
                    pts.append(o.encode(vec, float(self.mods[level]), o.qp_mods(level)))
                self.lts[ev["ret"]] = (idx, level, N1, pts)
                for r in self._lt_rotations(idx, N1):
                    self.galois_key(o.galois_element(r))
        for ev in self.trace["events"]:
            if ev["phase"] == "forward" and ev["op"] in ("RotateNew", "Rotate"):
                self.galois_key(o.galois_element(ev["args"][1]))

    def _lt_rotations(self, idx, N1):
        rots = set()
        for d in idx:
            rot = d & (self.slots - 1)
            rots.add(((rot // N1) * N1) & (self.slots - 1))
            rots.add(rot & (N1 - 1))
        return sorted(rots)

    # ---- input ----
    def encrypt(self, image):
        enc = [e for e in self.trace["events"] if e["phase"] == "input" and e["op"] == "Encode"][0]
        lvl, scale = enc["args"][1], enc["args"][2]
        v = np.zeros(self.slots)
        flat = np.asarray(image, dtype=np.float32).reshape(-1).astype(np.float64)
        v[:flat.size] = flat
        pt = self.orc.encode(v, float(scale), list(range(lvl + 1)))
        return (self.orc.encrypt_sk(self.seed + 3, self.sk, pt, lvl), lvl, float(scale))

    # ---- forward (the timed net(ct)) ----
    def _addmod(self, a, b, lvl):
        q = np.array(self.mods[:lvl + 1], dtype=np.uint64)[:, None]
        s = a + b
        return np.where(s >= q, s - q, s)

    def forward(self, ct_in):
        o = self.orc
        cts = {self.meta["input_ids"][0]: ct_in}
        for ev in self.trace["events"]:
            if ev["phase"] != "forward":
                continue
            op, a, ret = ev["op"], ev["args"], ev["ret"]
            if op in ("Decrypt", "Decode", "DeletePlaintext"):
                continue
            if op == "DeleteCiphertext":
                cts.pop(a[0], None)
                continue
            if op == "SetCiphertextScale":
                x, l, _ = cts[a[0]]
                cts[a[0]] = (x, l, float(a[1]))
                continue
            if op == "EvaluateLinearTransform":
                idx, level, N1, pts = self.lts[a[0]]
                x, l, s = cts[a[1]]
                lvl = min(l, level)
                gkeys = {}
                for r in self._lt_rotations(idx, N1):
                    g = o.galois_element(r)
                    gkeys[g] = self.galois_key(g)
                pts_l = [np.concatenate([p[:lvl + 1], p[level + 1:]]) for p in pts]
                y = o.lt_bsgs(np.ascontiguousarray(x[:, :lvl + 1]), lvl, idx, pts_l, N1, gkeys)
                cts[ret] = (y, lvl, s * self.mods[level])
            elif op in ("RescaleNew", "Rescale"):
                x, l, s = cts[a[0]]
                y = (o.rescale(x, l), l - 1, s / self.mods[l])
                cts[a[0]] = y
                cts[ret] = y
            elif op in ("RotateNew", "Rotate"):
                x, l, s = cts[a[0]]
                g = o.galois_element(a[1])
                cts[ret] = (o.rotate(x, g, self.galois_key(g), l), l, s)
            elif op in ("AddCiphertext", "AddCiphertextNew"):
                x, l, s = cts[a[0]]
                y, l2, _ = cts[a[1]]
                lv = min(l, l2)
                cts[ret] = (np.stack([self._addmod(x[c, :lv + 1], y[c, :lv + 1], lv) for c in range(2)]), lv, s)
            elif op in ("AddPlaintext", "AddPlaintextNew"):
                x, l, s = cts[a[0]]
                p, pl, _ = self.pts[a[1]]
                lv = min(l, pl)
                c0 = self._addmod(x[0, :lv + 1], p[:lv + 1], lv)
                cts[ret] = (np.stack([c0, x[1, :lv + 1]]), lv, s)
            elif op in ("MulRelinCiphertext", "MulRelinCiphertextNew"):
                x, l, s = cts[a[0]]
                y, l2, s2 = cts[a[1]]
                lv = min(l, l2)
                cts[ret] = (o.mul_relin(np.ascontiguousarray(x[:, :lv + 1]), np.ascontiguousarray(y[:, :lv + 1]),
                                        self.rlk, lv), lv, s * s2)
            else:
                raise RuntimeError(f"cpu replay: unsupported op {op}")
        return cts[self.meta["output_ids"][0]]

    def decrypt(self, ct):
        x, l, s = ct
        return self.orc.decode(self.orc.decrypt(x, self.sk, l), l, s)
