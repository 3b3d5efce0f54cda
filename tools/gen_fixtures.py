"""Generate the op-stream fixtures under tests/golden/ by driving the REFERENCE
Orion frontend (read-only at /root/reference) with a recording fake backend.

Runs only in the build container (the reference never travels to the GPU box).
Recipe: SURVEY.md Appendix B.  What it records is data: the exact sequence of
backend calls the reference's orion.nn / orion.core layers make for a model
(levels, scales, diagonal index sets and values, rotation amounts), plus the
cleartext model output for the same seeded input.  The GPU backend replays
this stream through its Lattigo-compatible C-ABI (orion_amd/replay.py).

Usage:  python tools/gen_fixtures.py lola_n15 [mlp_n14 ...]
"""
import json
import math
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")

CONFIGS = {
    # C3: LoLA at N=2^15: LogQ=[60]+[40]x11, LogP=[60,60]
    "lola_n15": dict(model="LoLA", logn=15, logq=[60] + [40] * 11, logp=[60, 60], logscale=40, h=192),
    # C2: MLP at N=2^14, 8 Q + 2 P primes
    "mlp_n14": dict(model="MLP", logn=14, logq=[60] + [40] * 7, logp=[60, 60], logscale=40, h=192),
    # C1 plumbing: configs/mlp.yml moduli sizes, Standard ring (SURVEY §7 note)
    "mlp_n13": dict(model="MLP", logn=13, logq=[29, 26, 26, 26, 26, 26], logp=[29, 29], logscale=26, h=8192),
    # C1 exactly as the reference's own test config tests/configs/mlp.yml (ConjugateInvariant ring:
    # N = 2^13 real slots, primes = 1 mod 4N)
    "mlp_n13_ci": dict(model="MLP", logn=13, logq=[29, 26, 26, 26, 26, 26], logp=[29, 29], logscale=26, h=8192,
                       ringtype="ConjugateInvariant"),
    # configs/lola.yml as written (ConjugateInvariant, N = 2^13, 26-bit chain)
    "lola_n13_ci": dict(model="LoLA", logn=13, logq=[29, 26, 26, 26, 26, 26], logp=[29, 29], logscale=26, h=8192,
                        ringtype="ConjugateInvariant"),
    # small LoLA for fast CPU/GPU end-to-end tests
    "lola_n13": dict(model="LoLA", logn=13, logq=[50] + [40] * 6, logp=[60, 60], logscale=40, h=192),
    # ResNet-20 (CIFAR-10) with the reference's configs/resnet.yml parameters (N=2^13, 30-bit chain,
    # bootstrapping); C4's ring degree is 2^16
    "resnet20_n13": dict(model="ResNet20", logn=13, logq=[60] + [30] * 32, logp=[60, 60], logscale=30, h=192,
                         boot_logp=[61] * 8, shape=(3, 32, 32), fuse=False),
    # C4 (BASELINE configs[3]): ResNet-20 at N=2^16 with the same moduli chain
    "resnet20_n16": dict(model="ResNet20", logn=16, logq=[60] + [30] * 32, logp=[60, 60], logscale=30, h=192,
                         boot_logp=[61] * 8, shape=(3, 32, 32), fuse=False),
}


def _tracer_shim():
    """The fork's StatsTracker.update_batch_size reads shape attributes off
    every traced module, including torch.nn.Identity (ResNet), which has none
    (orion/core/tracer.py:235-250): give such modules empty shapes."""
    import torch
    from orion.core import tracer

    orig = tracer.StatsTracker.update_batch_size

    def patched(self, batch_size):
        for node in self.module.graph.nodes:
            if node.op == "call_module":
                m = self.module.get_submodule(node.target)
                for a in ("input_shape", "output_shape", "fhe_input_shape", "fhe_output_shape"):
                    if not hasattr(m, a):
                        setattr(m, a, torch.Size([batch_size]))
        return orig(self, batch_size)

    tracer.StatsTracker.update_batch_size = patched


def _stub_modules():
    for name in ["h5py", "torchvision", "torchvision.datasets", "torchvision.transforms"]:
        sys.modules[name] = types.ModuleType(name)
    sys.modules["torchvision"].datasets = sys.modules["torchvision.datasets"]
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]


def _scipy_shim():
    import scipy.sparse
    import scipy.sparse._index as spi
    import torch

    def conv(x):
        if isinstance(x, torch.Tensor):
            return x.numpy()
        if isinstance(x, tuple):
            return tuple(conv(y) for y in x)
        return x

    orig_set = scipy.sparse.lil_matrix.__setitem__
    orig_get = spi.IndexMixin.__getitem__
    scipy.sparse.lil_matrix.__setitem__ = lambda self, k, v: orig_set(self, conv(k), conv(v))
    spi.IndexMixin.__getitem__ = lambda self, k: orig_get(self, conv(k))


class Recorder:
    """Fake backend: records every call the frontend makes (name, args, ret)."""

    def __init__(self, moduli, slots):
        self.moduli = moduli
        self.slots = slots
        self.events = []
        self.arrays = {}
        self.phase = "setup"
        self.pts, self.cts, self.lts, self.polys = {}, {}, {}, {}
        self._free = {"pt": [], "ct": [], "lt": [], "poly": []}
        self._next = {"pt": 0, "ct": 0, "lt": 0, "poly": 0}

    # lowest-free-id handle allocation (minheap.go:46-64)
    def _alloc(self, kind, meta):
        table = {"pt": self.pts, "ct": self.cts, "lt": self.lts, "poly": self.polys}[kind]
        if self._free[kind]:
            self._free[kind].sort()
            h = self._free[kind].pop(0)
        else:
            h = self._next[kind]
            self._next[kind] += 1
        table[h] = meta
        return h

    def _delete(self, kind, h):
        table = {"pt": self.pts, "ct": self.cts, "lt": self.lts}[kind]
        if h in table:
            del table[h]
            self._free[kind].append(h)

    def _rec(self, name, args, ret=None, arrays=None):
        ev = {"op": name, "args": args, "ret": ret, "phase": self.phase}
        if arrays:
            key = f"e{len(self.events)}"
            for k, v in arrays.items():
                self.arrays[f"{key}_{k}"] = v
            ev["arrays"] = key
        self.events.append(ev)
        return ret

    # ---- setup (no-ops, recorded) ------------------------------------
    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)

        def f(*args):
            return self._rec(name, [a if isinstance(a, (int, float, str)) else None for a in args])

        return f

    def GetModuliChain(self):
        return list(self.moduli)

    # ---- tensors ------------------------------------------------------
    def Encode(self, values, level, scale):
        h = self._alloc("pt", dict(level=level, scale=scale))
        return self._rec("Encode", [None, int(level), int(scale)], h,
                         {"values": np.asarray(values, dtype=np.float32)})

    def Decode(self, pid):
        self._rec("Decode", [pid])
        return [0.0] * self.slots

    def Encrypt(self, pid):
        p = self.pts[pid]
        h = self._alloc("ct", dict(level=p["level"], scale=p["scale"]))
        return self._rec("Encrypt", [pid], h)

    def Decrypt(self, cid):
        c = self.cts[cid]
        h = self._alloc("pt", dict(level=c["level"], scale=c["scale"]))
        return self._rec("Decrypt", [cid], h)

    def DeletePlaintext(self, h):
        self._delete("pt", h)
        return self._rec("DeletePlaintext", [h])

    def DeleteCiphertext(self, h):
        self._delete("ct", h)
        return self._rec("DeleteCiphertext", [h])

    def DeleteLinearTransform(self, h):
        h = int(h)
        self._delete("lt", h)
        return self._rec("DeleteLinearTransform", [h])

    def GetCiphertextScale(self, h):
        return self.cts[h]["scale"]

    def SetCiphertextScale(self, h, s):
        self.cts[h]["scale"] = int(s)
        return self._rec("SetCiphertextScale", [h, int(s)])

    def GetPlaintextScale(self, h):
        return self.pts[h]["scale"]

    def SetPlaintextScale(self, h, s):
        self.pts[h]["scale"] = int(s)
        return self._rec("SetPlaintextScale", [h, int(s)])

    def GetCiphertextLevel(self, h):
        return self.cts[h]["level"]

    def GetPlaintextLevel(self, h):
        return self.pts[h]["level"]

    def GetCiphertextSlots(self, h):
        return self.slots

    def GetPlaintextSlots(self, h):
        return self.slots

    def GetCiphertextDegree(self, h):
        return 1

    # ---- evaluator ----------------------------------------------------
    def _new_ct(self, name, args, level, scale):
        h = self._alloc("ct", dict(level=level, scale=scale))
        return self._rec(name, args, h)

    def RotateNew(self, c, k):
        m = self.cts[c]
        return self._new_ct("RotateNew", [c, int(k)], m["level"], m["scale"])

    def Rotate(self, c, k):
        return self._rec("Rotate", [c, int(k)], c)

    def RescaleNew(self, c):
        m = self.cts[c]
        return self._new_ct("RescaleNew", [c], m["level"] - 1, m["scale"] // self.moduli[m["level"]])

    def Rescale(self, c):
        m = self.cts[c]
        m["scale"] = m["scale"] // self.moduli[m["level"]]
        m["level"] -= 1
        return self._rec("Rescale", [c], c)

    def AddCiphertextNew(self, a, b):
        m = self.cts[a]
        return self._new_ct("AddCiphertextNew", [a, b], min(m["level"], self.cts[b]["level"]), m["scale"])

    def AddCiphertext(self, a, b):
        return self._rec("AddCiphertext", [a, b], a)

    def SubCiphertextNew(self, a, b):
        m = self.cts[a]
        return self._new_ct("SubCiphertextNew", [a, b], m["level"], m["scale"])

    def SubCiphertext(self, a, b):
        return self._rec("SubCiphertext", [a, b], a)

    def AddPlaintextNew(self, a, p):
        m = self.cts[a]
        return self._new_ct("AddPlaintextNew", [a, p], m["level"], m["scale"])

    def AddPlaintext(self, a, p):
        return self._rec("AddPlaintext", [a, p], a)

    def SubPlaintext(self, a, p):
        return self._rec("SubPlaintext", [a, p], a)

    def MulPlaintextNew(self, a, p):
        m = self.cts[a]
        return self._new_ct("MulPlaintextNew", [a, p], m["level"], m["scale"] * self.pts[p]["scale"])

    def MulPlaintext(self, a, p):
        self.cts[a]["scale"] *= self.pts[p]["scale"]
        return self._rec("MulPlaintext", [a, p], a)

    def MulRelinCiphertextNew(self, a, b):
        m = self.cts[a]
        return self._new_ct("MulRelinCiphertextNew", [a, b], min(m["level"], self.cts[b]["level"]),
                            m["scale"] * self.cts[b]["scale"])

    def MulRelinCiphertext(self, a, b):
        self.cts[a]["scale"] *= self.cts[b]["scale"]
        return self._rec("MulRelinCiphertext", [a, b], a)

    def AddScalar(self, a, s):
        return self._rec("AddScalar", [a, float(s)], a)

    def AddScalarNew(self, a, s):
        m = self.cts[a]
        return self._new_ct("AddScalarNew", [a, float(s)], m["level"], m["scale"])

    def MulScalarInt(self, a, s):
        return self._rec("MulScalarInt", [a, int(s)], a)

    def MulScalarIntNew(self, a, s):
        m = self.cts[a]
        return self._new_ct("MulScalarIntNew", [a, int(s)], m["level"], m["scale"])

    def MulScalarFloat(self, a, s):
        self.cts[a]["scale"] *= self.moduli[self.cts[a]["level"]]
        return self._rec("MulScalarFloat", [a, float(s)], a)

    def MulScalarFloatNew(self, a, s):
        m = self.cts[a]
        return self._new_ct("MulScalarFloatNew", [a, float(s)], m["level"], m["scale"] * self.moduli[m["level"]])

    def Negate(self, a):
        m = self.cts[a]
        return self._new_ct("Negate", [a], m["level"], m["scale"])

    # ---- polynomials (polyeval.go) and bootstrapping (bootstrapper.go) ----------
    def GenerateMinimaxSignCoeffs(self, degrees, prec, logalpha, logerr, debug):
        # the coefficients come from this build's generator (host code, CPU): Lattigo's composite
        # construction restated [U] and pinned to the prec-bit mpmath computation of the same
        # (tools/gen_minimax.py -> tests/golden/minimax_sign.json, tests/test_minimax.py)
        from orion_amd.backend import HipLibrary
        out = HipLibrary().GenerateMinimaxSignCoeffs(list(degrees), prec, logalpha, logerr, debug)
        self._rec("GenerateMinimaxSignCoeffs", [list(map(int, degrees)), int(prec), int(logalpha), int(logerr)])
        return out

    def _poly(self, name, coeffs):
        c = np.asarray(coeffs, dtype=np.float32)
        h = self._alloc("poly", dict(n=len(c)))
        return self._rec(name, [None], h, {"coeffs": c})

    def GenerateMonomial(self, coeffs, *rest):
        return self._poly("GenerateMonomial", coeffs)

    def GenerateChebyshev(self, coeffs, *rest):
        return self._poly("GenerateChebyshev", coeffs)

    def EvaluatePolynomial(self, c, p, out_scale):
        m = self.cts[c]
        depth = int(self.polys[p]["n"] - 1).bit_length()
        return self._new_ct("EvaluatePolynomial", [c, p, int(out_scale)], m["level"] - depth, int(out_scale))

    def NewBootstrapper(self, logp, slots):
        return self._rec("NewBootstrapper", [None, int(slots)])

    def Bootstrap(self, c, slots):
        m = self.cts[c]
        return self._new_ct("Bootstrap", [c, int(slots)], len(self.moduli) - 1, m["scale"])

    # ---- linear transforms ------------------------------------------------
    def GenerateLinearTransform(self, idxs, data, level, ratio, io_mode):
        h = self._alloc("lt", dict(level=level, idxs=list(idxs), ratio=float(ratio)))
        return self._rec("GenerateLinearTransform", [list(map(int, idxs)), None, int(level), float(ratio), io_mode], h,
                         {"diags": np.asarray(data, dtype=np.float32).reshape(len(idxs), self.slots)})

    def GetLinearTransformRotationKeys(self, h):
        # galois elements are resolved by the backend itself at replay time
        return [("lt", h)]

    def GenerateConsolidatedRotationKeys(self, keys):
        return self._rec("GenerateConsolidatedRotationKeys", [None])

    def EvaluateLinearTransform(self, t, c):
        t, c = int(t), int(c)
        m = self.cts[c]
        lt = self.lts[t]
        return self._new_ct("EvaluateLinearTransform", [t, c], min(m["level"], lt["level"]),
                            m["scale"] * self.moduli[lt["level"]])


def run(name):
    import torch

    cfg = CONFIGS[name]
    sys.path.insert(0, REF)
    sys.dont_write_bytecode = True
    _stub_modules()
    _scipy_shim()
    import orion
    import orion.models as models
    from orion.core import orion as core
    _tracer_shim()

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from oracle.oracle import gen_moduli  # primes for GetModuliChain (frontend uses them)

    ci = cfg.get("ringtype", "standard").lower() == "conjugateinvariant"
    # parameters.py:33-36: logslots = logn (ConjugateInvariant) or logn - 1; the CI ring's NthRoot is 4N
    moduli = gen_moduli(cfg["logn"] + ci, cfg["logq"], cfg["logp"])
    slots = 1 << (cfg["logn"] - 1 + ci)
    rec = Recorder(moduli[: len(cfg["logq"])], slots)
    core.Scheme.setup_backend = lambda self, params: rec

    torch.manual_seed(42)
    conf = {
        "ckks_params": {"LogN": cfg["logn"], "LogQ": cfg["logq"], "LogP": cfg["logp"],
                        "LogScale": cfg["logscale"], "H": cfg["h"],
                        "RingType": cfg.get("ringtype", "Standard")},
        "boot_params": {"LogP": cfg.get("boot_logp", [61] * 2)},
        "orion": {"margin": 2, "embedding_method": "hybrid", "backend": "lattigo",
                  "fuse_modules": cfg.get("fuse", True), "debug": False, "diags_path": "", "keys_path": "",
                  "io_mode": "none"},
    }
    orion.init_scheme(conf)
    net = getattr(models, cfg["model"])()
    net.eval()
    from torch.utils.data import DataLoader, TensorDataset
    shape = cfg.get("shape", (1, 28, 28))
    nfit = 256 if shape == (1, 28, 28) else 32
    fit_imgs = torch.randn(nfit, *shape)
    fit_data = DataLoader(TensorDataset(fit_imgs, torch.zeros(nfit)), batch_size=1)
    inp = torch.randn(1, *shape)
    out_clear = net(inp).detach()
    orion.fit(net, fit_data)
    rec.phase = "compile"
    input_level = orion.compile(net)
    rec.phase = "input"
    vec_ptxt = orion.encode(inp, input_level)
    vec_ctxt = orion.encrypt(vec_ptxt)
    net.he()
    rec.phase = "forward"
    out_ctxt = net(vec_ctxt)
    rec.phase = "output"
    out_ctxt.decrypt()
    rec.phase = "done"

    meta = dict(name=name, config=cfg, moduli=moduli, slots=slots, input_level=input_level,
                input_ids=vec_ctxt.ids, output_ids=out_ctxt.ids,
                output_shape=list(out_clear.shape), reference="AdrianHeath988/orion @ /root/reference",
                generator="tools/gen_fixtures.py (reference frontend + recording backend)")
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"{name}_trace.json"), "w") as f:
        json.dump({"meta": meta, "events": rec.events}, f, indent=0,
                  default=lambda o: int(o) if isinstance(o, np.integer) else float(o))
    arrays = dict(rec.arrays)
    arrays["input"] = inp.numpy().astype(np.float32)
    arrays["expected_output"] = out_clear.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(OUT, f"{name}_arrays.npz"), **arrays)
    counts = {}
    for e in rec.events:
        if e["phase"] == "forward":
            counts[e["op"]] = counts.get(e["op"], 0) + 1
    print(name, "input level", input_level, "forward ops:", counts)


if __name__ == "__main__":
    for n in sys.argv[1:] or ["lola_n15"]:
        run(n)
