"""Replay an Orion op stream through the HIP backend's Lattigo-compatible API.

The stream (tests/golden/<name>_trace.json + _arrays.npz) is the exact
sequence of backend calls the reference frontend makes for a model
(orion/nn/*.py -> orion/backend/python/*.py -> backend), recorded by
tools/gen_fixtures.py.  Replaying it here reproduces `net(ct)` of
/root/reference/examples/run_lola.py:45-47 call for call, with two
deliberate differences:

* the fork's debug decryptions inside the forward pass
  (lt_evaluator.py:156-158,194-196; activation.py:51-62) are skipped -- they
  need the secret key and are not part of the operator semantics;
* one ciphertext handle carries a batch of B images (EncodeBatch), so every
  call of the stream runs once for the whole batch.

Handles recorded in the trace are mapped to the library's own handles at the
events that create them, so deletes and lowest-free-id reuse replay exactly.
Every other call goes through its own C-ABI entry, in the stream's order: the
rotate-and-add fusion of `out += out.roll(k)` (RotateNew, AddCiphertext,
DeleteCiphertext) and RescaleNew's copy-on-write result happen inside the
library, behind the unchanged calls (backend.hip Context::Deferred, alias).

Concurrency is the frontend's own: several threads each call forward() of the
same compiled stream on ciphertexts they encrypted themselves (Pipelines).
With thread pipelines on (OrionHipThreadPipelines) the library gives each
thread a context of its own -- the scheme's keys and compiled objects, its own
HIP stream, pool and handles -- so the threads' kernels overlap on the GPU.
forward() keeps its state in locals, so it is reentrant across threads.
"""
import json
import os
import queue
import threading

import numpy as np

from .backend import HipLibrary

GOLDEN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def load_stream(name, root=GOLDEN):
    with open(os.path.join(root, f"{name}_trace.json")) as f:
        trace = json.load(f)
    arrays = dict(np.load(os.path.join(root, f"{name}_arrays.npz"), allow_pickle=False))
    return trace, arrays


# ops whose trace args are (ct, ct|pt|scalar) and that return a ciphertext
_CT_OPS = {
    "RotateNew": ("ct", "int"), "Rotate": ("ct", "int"),
    "RescaleNew": ("ct",), "Rescale": ("ct",),
    "AddCiphertext": ("ct", "ct"), "AddCiphertextNew": ("ct", "ct"),
    "SubCiphertext": ("ct", "ct"), "SubCiphertextNew": ("ct", "ct"),
    "MulRelinCiphertext": ("ct", "ct"), "MulRelinCiphertextNew": ("ct", "ct"),
    "AddPlaintext": ("ct", "pt"), "AddPlaintextNew": ("ct", "pt"),
    "SubPlaintext": ("ct", "pt"), "SubPlaintextNew": ("ct", "pt"),
    "MulPlaintext": ("ct", "pt"), "MulPlaintextNew": ("ct", "pt"),
    "AddScalar": ("ct", "float"), "AddScalarNew": ("ct", "float"),
    "SubScalar": ("ct", "float"), "SubScalarNew": ("ct", "float"),
    "MulScalarInt": ("ct", "int"), "MulScalarIntNew": ("ct", "int"),
    "MulScalarFloat": ("ct", "float"), "MulScalarFloatNew": ("ct", "float"),
    "Negate": ("ct",),
    "EvaluateLinearTransform": ("lt", "ct"),
    "EvaluatePolynomial": ("ct", "poly", "int"),
    "Bootstrap": ("ct", "int"),
}
# ops that allocate a new ciphertext handle
_NEW_CT = ("EvaluateLinearTransform", "EvaluatePolynomial", "Bootstrap", "Negate")


class OrionStream:
    """A compiled Orion model as an op stream bound to one HipLibrary."""

    def __init__(self, name, lib=None, seed=2024, device=None, root=GOLDEN, synthetic_diagonals=False):
        self.name = name
        self.trace, self.arrays = load_stream(name, root)
        self.meta = self.trace["meta"]
        cfg = self.meta["config"]
        self.lib = lib or HipLibrary()
        self.lib.new_scheme(cfg["logn"], cfg["logq"], cfg["logp"], cfg["logscale"], h=cfg["h"], seed=seed,
                            device=device, ringtype=cfg.get("ringtype", "standard"))
        self.slots = self.meta["slots"]
        self.synthetic = synthetic_diagonals
        self.pt_map, self.ct_map, self.lt_map, self.poly_map = {}, {}, {}, {}
        self.input_level = self.meta["input_level"]
        self._events = self.trace["events"]

    # -- setup: keys + evaluator (key_generator.py:10-15, evaluator.py:2-6) ---
    def keygen(self, with_po2=True):
        lib = self.lib
        lib.NewKeyGenerator()
        lib.GenerateSecretKey()
        lib.GeneratePublicKey()
        lib.GenerateRelinearizationKey()
        lib.GenerateEvaluationKeys()
        lib.NewEncoder()
        lib.NewEncryptor()
        lib.NewDecryptor()
        if with_po2:
            lib.NewEvaluator()  # power-of-two rotation keys (evaluator.go:25-31)
        lib.NewPolynomialEvaluator()
        lib.NewLinearTransformEvaluator()

    # -- compile phase: bias plaintexts + linear transforms + their keys --------
    def compile(self, gen_keys=True):
        lib = self.lib
        rng = np.random.default_rng(7)
        for ev in self._events:
            if ev["phase"] != "compile":
                continue
            op, args, ret = ev["op"], ev["args"], ev["ret"]
            if op == "Encode":
                vals = self.arrays[ev["arrays"] + "_values"]
                self.pt_map[ret] = lib.Encode(vals, args[1], args[2])
            elif op == "GenerateLinearTransform":
                idx, _, level, ratio, io = args
                diags = self.arrays[ev["arrays"] + "_diags"]
                if self.synthetic:
                    diags = rng.uniform(-1, 1, diags.shape).astype(np.float32)
                h = lib.GenerateLinearTransform(idx, diags.reshape(-1), level, ratio, "none")
                self.lt_map[ret] = h
                if gen_keys:
                    lib.GenerateConsolidatedRotationKeys(lib.GetLinearTransformRotationKeys(h))
            elif op == "DeletePlaintext" and args[0] in self.pt_map:
                lib.DeletePlaintext(self.pt_map.pop(args[0]))
            elif op in ("GenerateChebyshev", "GenerateMonomial"):  # poly_evaluator.py:15-23
                coeffs = self.arrays[ev["arrays"] + "_coeffs"]
                self.poly_map[ret] = (lib.GenerateChebyshev(list(coeffs), len(coeffs)) if op == "GenerateChebyshev"
                                      else lib.GenerateMonomial(list(coeffs)))
            elif op == "NewBootstrapper":  # bootstrapper.py:9-13 (boot_logp of the config)
                lib.NewBootstrapper(list(self.meta["config"].get("boot_logp") or []), args[1])
        # rotation amounts used by the forward pass (hybrid output rotations)
        if gen_keys:
            for ev in self._events:
                if ev["phase"] == "forward" and ev["op"] in ("RotateNew", "Rotate"):
                    lib.AddRotationKey(ev["args"][1])

    def input_events(self):
        return [e for e in self._events if e["phase"] == "input"]

    # -- input phase: encode + encrypt a batch of images -------------------------
    def encrypt_batch(self, images):
        """images: (B, ...) array; each image flattened into the slots the way
        orion's encoder pads it (encoder.py:29-42)."""
        imgs = np.asarray(images, dtype=np.float32).reshape(len(images), -1)
        enc = [e for e in self.input_events() if e["op"] == "Encode"][0]
        level, scale = enc["args"][1], enc["args"][2]
        vals = np.zeros((imgs.shape[0], self.slots), dtype=np.float32)
        vals[:, :imgs.shape[1]] = imgs
        pt = self.lib.encode_batch(vals, level, scale)
        ct = self.lib.Encrypt(pt)
        self.lib.DeletePlaintext(pt)
        return ct

    def reference_input(self):
        return self.arrays["input"]

    # -- forward: the timed net(ct) ------------------------------------------------
    def forward(self, ct_in, hook=None, stop_after=None):
        """hook(event, handle): called after every replayed op (debugging).
        stop_after: index of a forward event; the handle that event produced is
        returned (the stream's other temporaries are deleted)."""
        it = self.forward_iter(ct_in, hook, stop_after)
        while True:
            try:
                next(it)
            except StopIteration as e:
                return e.value

    def forward_iter(self, ct_in, hook=None, stop_after=None):
        """forward() one op at a time: yields after every library call that
        enqueues GPU work; the generator's return value is the output."""
        lib = self.lib
        in_ids = self.meta["input_ids"]
        ct_map = {in_ids[0]: ct_in}
        skipped_pts = set()
        owned = set()
        fi = -1
        for ev in self._events:
            if ev["phase"] != "forward":
                continue
            fi += 1
            op, args, ret = ev["op"], ev["args"], ev["ret"]
            if op in ("Decrypt", "Decode"):  # debug decryptions of the fork: not operator semantics
                if op == "Decrypt":
                    skipped_pts.add(ret)
                continue
            if op == "DeletePlaintext":
                if args[0] in skipped_pts:
                    skipped_pts.discard(args[0])
                elif args[0] in self.pt_map:
                    lib.DeletePlaintext(self.pt_map.pop(args[0]))
                continue
            if op == "DeleteCiphertext":
                h = ct_map.pop(args[0], None)
                if h is not None and h in owned:
                    lib.DeleteCiphertext(h)
                    owned.discard(h)
                continue
            if op == "SetCiphertextScale":
                lib.SetCiphertextScale(ct_map[args[0]], args[1])
                continue
            kinds = _CT_OPS.get(op)
            if kinds is None:
                raise RuntimeError(f"replay: unsupported op {op} in forward phase")
            cargs = []
            for k, a in zip(kinds, args):
                cargs.append(ct_map[a] if k == "ct" else self.pt_map[a] if k == "pt" else
                             self.lt_map[a] if k == "lt" else self.poly_map[a] if k == "poly" else a)
            h = getattr(lib, op)(*cargs)
            yield
            if hook is not None:
                hook(ev, h)
            if ret is not None:
                if op.endswith("New") or op in _NEW_CT:
                    owned.add(h)
                ct_map[ret] = h
            if stop_after is not None and fi == stop_after:
                break
        out = ct_map[ret] if stop_after is not None else ct_map[self.meta["output_ids"][0]]
        for rid, h in ct_map.items():
            if h != out and h in owned:
                lib.DeleteCiphertext(h)
        return out

    def capture(self, ct_in):
        """Record forward(clone(ct_in)) into one hipGraph (OrionHipGraphBegin/End):
        returns (graph id, output handle).  Each OrionHipGraphLaunch(graph)
        re-runs every kernel of the pass on ct_in's current contents and
        rewrites the output handle; the clone keeps in-place ops off ct_in.
        Run forward() once first (keys, tables and LT plans are made then)."""
        lib = self.lib
        lib.OrionHipGraphBegin()
        try:
            x = lib.CloneCiphertext(ct_in)
            out = self.forward(x)
            if out != x:
                lib.DeleteCiphertext(x)
        except Exception:
            try:
                lib.OrionHipGraphEnd()
            except RuntimeError:
                pass
            raise
        return lib.OrionHipGraphEnd(), out

    def decrypt_output(self, ct, n_out=None):
        """Decrypt + decode a batch output; returns (B, n_out) floats."""
        lib = self.lib
        B = lib.GetCiphertextBatch(ct)
        pt = lib.Decrypt(ct)
        vals = np.array(lib.Decode(pt), dtype=np.float64).reshape(B, self.slots)
        lib.DeletePlaintext(pt)
        n = n_out or int(np.prod(self.meta["output_shape"]))
        return vals[:, :n]

    def forward_op_counts(self):
        c = {}
        for e in self._events:
            if e["phase"] == "forward" and e["op"] not in ("Decrypt", "Decode", "DeletePlaintext",
                                                          "DeleteCiphertext"):
                c[e["op"]] = c.get(e["op"], 0) + 1
        return c


class Pipelines:
    """n worker threads, each bound by the library to a pipeline context of its
    own at its first call (OrionHipThreadPipelines(n + 1): the scheme's context
    plus n).  run(fns) runs fns[i] on thread i and returns the results in
    order; a worker's exception is raised in the caller.  The threads keep
    their contexts (and the handles made there) across run() calls."""

    def __init__(self, lib, n, device=None):
        self.lib, self.n = lib, n
        self.prev = lib.thread_pipelines(n + 1)
        self._tasks = [queue.Queue() for _ in range(n)]
        self._done = queue.Queue()
        self._threads = [threading.Thread(target=self._work, args=(i, device), daemon=True) for i in range(n)]
        for t in self._threads:
            t.start()
        self.contexts = self.run([self.lib.OrionHipCurrentPipeline] * n)

    def _work(self, i, device):
        if device is not None:
            import torch
            torch.cuda.set_device(device)
        while True:
            fn = self._tasks[i].get()
            if fn is None:
                return
            try:
                self._done.put((i, True, fn()))
            except BaseException as e:  # reported by run()
                self._done.put((i, False, e))

    def run(self, fns):
        assert len(fns) == self.n
        for q, fn in zip(self._tasks, fns):
            q.put(fn)
        out, err = [None] * self.n, None
        for _ in range(self.n):
            i, ok, v = self._done.get()
            if ok:
                out[i] = v
            elif err is None:
                err = v
        if err is not None:
            raise err
        return out

    def run_one(self, i, fn):
        """fn on thread i alone (the others idle)."""
        fns = [(lambda: None)] * self.n
        fns[i] = fn
        return self.run(fns)[i]

    def close(self):
        for q in self._tasks:
            q.put(None)
        for t in self._threads:
            t.join()
        self.lib.thread_pipelines(self.prev)
