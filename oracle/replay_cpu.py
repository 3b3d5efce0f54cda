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
        self.polys = {}  # handle -> (coefficients, chebyshev)
        self.bootstrappers = {}  # slots -> (bootstrapping-chain Oracle, oracle.BtpCircuit, keys)

    # ---- keys ----
    def keygen(self):
        o = self.orc
        self.sk = o.gen_secret(self.seed, self.h)
        s2 = o.mul_coeffs(self.sk, self.sk, list(range(self.L + self.K)))
        self.rlk = o.gen_evk(self.seed + 1, s2, self.sk)

    key_source = None  # optional callable galEl -> evk (keys shared from another backend)

    def galois_key(self, g):
        if g not in self.gks and self.key_source is not None:
            self.gks[g] = self.key_source(g)
        if g not in self.gks:
            M = (4 if self.ci else 2) * self.N  # NthRoot
            ginv = pow(g, -1, M)
            s_out = self.orc.automorphism_ntt(self.sk, ginv)
            self.gks[g] = self.orc.gen_evk(self.seed + 7 + len(self.gks), self.sk, s_out)
        return self.gks[g]

    # ---- compile ----
    # Plaintexts and transforms are encoded on first use, and with keys=False
    # no Galois key is made up front (galois_key then fetches or generates it
    # when a forward op needs it): a replay of a prefix of a large stream
    # (ResNet-20) touches only what the prefix uses.
    def compile(self, keys=True, lazy=False):
        o = self.orc
        for ev in self.trace["events"]:
            if ev["phase"] != "compile":
                continue
            if ev["op"] == "Encode":
                lvl, scale = ev["args"][1], ev["args"][2]
                self.pts[ev["ret"]] = ("lazy", ev["arrays"] + "_values", lvl, scale)
            elif ev["op"] in ("GenerateChebyshev", "GenerateMonomial"):
                coeffs = self.arrays[ev["arrays"] + "_coeffs"].astype(np.float32).astype(np.float64)
                self.polys[ev["ret"]] = (coeffs, ev["op"] == "GenerateChebyshev")
            elif ev["op"] == "GenerateLinearTransform":
                idx, _, level, ratio, _ = ev["args"]
                import math
                N1 = o.find_best_bsgs_n1(idx, int(math.log(ratio)))
                self.lts[ev["ret"]] = ("lazy", ev["arrays"] + "_diags", idx, level, N1)
                if keys:
                    for r in self._lt_rotations(idx, N1):
                        self.galois_key(o.galois_element(r))
        if keys:
            for ev in self.trace["events"]:
                if ev["phase"] == "forward" and ev["op"] in ("RotateNew", "Rotate"):
                    self.galois_key(o.galois_element(ev["args"][1]))
        if not lazy:  # everything encoded now (the CPU baseline times forward() alone)
            for h in list(self.pts):
                self._pt(h)
            for h in list(self.lts):
                self._lt(h)

    def _pt(self, h):
        p = self.pts[h]
        if isinstance(p[0], str):
            _, name, lvl, scale = p
            vals = self.arrays[name].astype(np.float64)
            p = self.pts[h] = (self.orc.encode(vals, float(scale), list(range(lvl + 1))), lvl, np.longdouble(int(scale)))
        return p

    def _lt(self, h):
        t = self.lts[h]
        if isinstance(t[0], str):
            _, name, idx, level, N1 = t
            o = self.orc
            diags = self.arrays[name].astype(np.float64)
            pts = []
            for i, d in enumerate(idx):
                rot = d & (self.slots - 1)
                giant = ((rot // N1) * N1) & (self.slots - 1)
                vec = np.roll(diags[i], giant)  # right rotation by the giant step
                pts.append(o.encode(vec, float(self.mods[level]), o.qp_mods(level)))
            t = self.lts[h] = (idx, level, N1, pts)
        return t

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
    # Scales are tracked as 80-bit long doubles (numpy longdouble), as the HIP
    # backend's host code tracks them: products like 2^30 q_l are not exact in
    # float64, and the polynomial evaluator rounds its constants against them.
    def _addmod(self, a, b, lvl):
        q = np.array(self.mods[:lvl + 1], dtype=np.uint64)[:, None]
        s = a + b
        return np.where(s >= q, s - q, s)

    def _submod(self, a, b, lvl):
        q = np.array(self.mods[:lvl + 1], dtype=np.uint64)[:, None]
        return np.where(a >= b, a - b, a + q - b)

    def _mulconst(self, x, k, lvl):
        """x [..][lvl+1][N] times the per-limb constants k (python ints)."""
        o = self.orc
        mods = list(range(lvl + 1))
        kk = np.stack([np.full(self.N, int(k[j]) % self.mods[j], dtype=np.uint64) for j in mods])
        if x.ndim == 2:
            return o.mul_coeffs(np.ascontiguousarray(x[:lvl + 1]), kk, mods)
        return np.stack([o.mul_coeffs(np.ascontiguousarray(x[c, :lvl + 1]), kk, mods) for c in range(x.shape[0])])

    @staticmethod
    def _round_away(x):
        """round half away from zero of a longdouble, as a python int"""
        x = np.longdouble(x)
        a = np.floor(abs(x) + np.longdouble(0.5))
        r = int(a)
        return -r if x < 0 else r

    def _const(self, v, lvl):
        return [int(v) % self.mods[j] for j in range(lvl + 1)]

    def _add_like(self, x, l, s, y, yl, ys, ncomp_y, sub):
        """backend.hip Context::add_like (Lattigo evaluateInPlace scale matching)"""
        lv = min(l, yl)
        x = x[:, :lv + 1]
        y = y[:ncomp_y, :lv + 1] if y.ndim == 3 else y[None, :lv + 1]
        ratio = s / ys if s > ys else ys / s
        r = self._round_away(ratio)
        op = self._submod if sub else self._addmod
        out_s = s
        if r > 1:
            k = self._const(r, lv)
            if s > ys:
                y = self._mulconst(y, k, lv)
            else:
                x = self._mulconst(x, k, lv)
                out_s = ys
        out = x.copy()
        for c in range(y.shape[0]):
            out[c] = op(x[c], y[c], lv)
        return (out, lv, out_s)

    def forward(self, ct_in, stop_after=None):
        """ct_in = (ct [2][l+1][N], level, scale).  stop_after: index of a
        forward event; the ciphertext that event produced is returned."""
        o = self.orc
        LD = np.longdouble
        x0, l0, s0 = ct_in
        cts = {self.meta["input_ids"][0]: (x0, l0, LD(s0))}
        fi = -1
        for ev in self.trace["events"]:
            if ev["phase"] != "forward":
                continue
            fi += 1
            op, a, ret = ev["op"], ev["args"], ev["ret"]
            if op in ("Decrypt", "Decode", "DeletePlaintext"):
                continue
            if op == "DeleteCiphertext":
                cts.pop(a[0], None)
                continue
            if op == "SetCiphertextScale":
                x, l, _ = cts[a[0]]
                cts[a[0]] = (x, l, LD(a[1]))
                continue
            if op == "EvaluateLinearTransform":
                idx, level, N1, pts = self._lt(a[0])
                x, l, s = cts[a[1]]
                lvl = min(l, level)
                gkeys = {}
                for r in self._lt_rotations(idx, N1):
                    g = o.galois_element(r)
                    if g != 1:  # the zero rotation needs no key
                        gkeys[g] = self.galois_key(g)
                pts_l = [np.concatenate([p[:lvl + 1], p[level + 1:]]) for p in pts]
                y = o.lt_bsgs(np.ascontiguousarray(x[:, :lvl + 1]), lvl, idx, pts_l, N1, gkeys)
                cts[ret] = (y, lvl, s * LD(self.mods[level]))
            elif op in ("RescaleNew", "Rescale"):
                x, l, s = cts[a[0]]
                y = (o.rescale(np.ascontiguousarray(x[:, :l + 1]), l), l - 1, s / LD(self.mods[l]))
                cts[a[0]] = y
                cts[ret] = y
            elif op in ("RotateNew", "Rotate"):
                x, l, s = cts[a[0]]
                g = o.galois_element(a[1])
                cts[ret] = (o.rotate(np.ascontiguousarray(x[:, :l + 1]), g, self.galois_key(g), l), l, s)
            elif op in ("AddCiphertext", "AddCiphertextNew", "SubCiphertext", "SubCiphertextNew"):
                x, l, s = cts[a[0]]
                y, l2, s2 = cts[a[1]]
                cts[ret] = self._add_like(x, l, s, y, l2, s2, 2, op.startswith("Sub"))
            elif op in ("AddPlaintext", "AddPlaintextNew", "SubPlaintext", "SubPlaintextNew"):
                x, l, s = cts[a[0]]
                p, pl, ps = self._pt(a[1])
                cts[ret] = self._add_like(x, l, s, p, pl, LD(ps), 1, op.startswith("Sub"))
            elif op in ("MulPlaintext", "MulPlaintextNew"):
                x, l, s = cts[a[0]]
                p, pl, ps = self._pt(a[1])
                lv = min(l, pl)
                mods = list(range(lv + 1))
                y = np.stack([o.mul_coeffs(np.ascontiguousarray(x[c, :lv + 1]), np.ascontiguousarray(p[:lv + 1]), mods)
                              for c in range(2)])
                cts[ret] = (y, lv, s * LD(ps))
            elif op in ("MulRelinCiphertext", "MulRelinCiphertextNew"):
                x, l, s = cts[a[0]]
                y, l2, s2 = cts[a[1]]
                lv = min(l, l2)
                cts[ret] = (o.mul_relin(np.ascontiguousarray(x[:, :lv + 1]), np.ascontiguousarray(y[:, :lv + 1]),
                                        self.rlk, lv), lv, s * s2)
            elif op in ("AddScalar", "AddScalarNew", "SubScalar", "SubScalarNew"):
                x, l, s = cts[a[0]]
                v = np.float32(a[1]) * (-1 if op.startswith("Sub") else 1)
                k = self._const(self._round_away(LD(float(v)) * s), l)
                y = x[:, :l + 1].copy()
                kk = np.array(k, dtype=np.uint64)[:, None]
                y[0] = self._addmod(y[0], np.broadcast_to(kk, y[0].shape), l)
                cts[ret] = (y, l, s)
            elif op in ("MulScalarInt", "MulScalarIntNew"):
                x, l, s = cts[a[0]]
                cts[ret] = (self._mulconst(x[:, :l + 1], self._const(int(a[1]), l), l), l, s)
            elif op in ("MulScalarFloat", "MulScalarFloatNew"):
                x, l, s = cts[a[0]]
                dv = float(np.float32(a[1]))
                if dv == np.floor(dv):
                    cts[ret] = (self._mulconst(x[:, :l + 1], self._const(int(dv), l), l), l, s)
                else:
                    ql = LD(self.mods[l])
                    r = self._round_away(LD(dv) * ql)
                    cts[ret] = (self._mulconst(x[:, :l + 1], self._const(r, l), l), l, s * ql)
            elif op == "EvaluatePolynomial":
                x, l, s = cts[a[0]]
                coeffs, cheb = self.polys[a[1]]
                y, lv, sc = o.eval_poly_ld(np.ascontiguousarray(x[:, :l + 1]), l, s, coeffs, cheb, LD(a[2]), self.rlk)
                cts[ret] = (y, lv, sc)
            elif op == "Bootstrap":
                x, l, s = cts[a[0]]
                boot, circ, keys = self.bootstrappers[a[1]]
                y, ys = o.bootstrap(boot, circ, keys, np.ascontiguousarray(x[:, :l + 1]), l, s)
                cts[ret] = (y, self.L - 1, LD(ys))
            else:
                raise RuntimeError(f"cpu replay: unsupported op {op}")
            if stop_after is not None and fi == stop_after:
                return cts[ret]
        return cts[self.meta["output_ids"][0]]

    def decrypt(self, ct):
        x, l, s = ct
        return self.orc.decode(self.orc.decrypt(x, self.sk, l), l, s)
