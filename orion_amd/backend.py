"""Python binding of liborion_hip.so -- the MI355X backend behind Orion's
backend-plugin API.

`HipLibrary` mirrors the reference's `LattigoLibrary`
(/root/reference/orion/backend/lattigo/bindings.py:94-746): same method names,
argument meaning (handles are ints, scalars/diagonals cross as C float,
scales as unsigned long) and list conversions, so Orion's L1 wrappers
(orion/backend/python/*.py) can drive it unchanged.  A maintainer selects it
in `Scheme.setup_backend` (orion/core/orion.py:90-106) -- see INTEGRATION.md.

Error behaviour: the library never aborts; failed calls raise RuntimeError
with the library's message (Lattigo would panic and abort the process).

This module never falls back to a CPU implementation: if the HIP extension
cannot be loaded, or no GPU is visible when the scheme is created, it raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ORION_LIB") or os.path.join(_HERE, "liborion_hip.so")

c_int, c_float, c_ulong, c_double, c_char_p, c_void_p = (
    ctypes.c_int, ctypes.c_float, ctypes.c_ulong, ctypes.c_double, ctypes.c_char_p, ctypes.c_void_p)
P = ctypes.POINTER


class ArrayResultInt(ctypes.Structure):
    _fields_ = [("Data", P(ctypes.c_int)), ("Length", ctypes.c_ulong)]


class ArrayResultFloat(ctypes.Structure):
    _fields_ = [("Data", P(ctypes.c_float)), ("Length", ctypes.c_ulong)]


class ArrayResultDouble(ctypes.Structure):
    _fields_ = [("Data", P(ctypes.c_double)), ("Length", ctypes.c_ulong)]


class ArrayResultUInt64(ctypes.Structure):
    _fields_ = [("Data", P(ctypes.c_ulong)), ("Length", ctypes.c_ulong)]


class ArrayResultByte(ctypes.Structure):
    _fields_ = [("Data", P(ctypes.c_ubyte)), ("Length", ctypes.c_ulong)]


# name -> (argtypes, restype); the Lattigo-compatible set first
SIGNATURES = {
    "NewScheme": ([c_int, P(c_int), c_int, P(c_int), c_int, c_int, c_int, c_char_p, c_char_p, c_char_p], None),
    "DeleteScheme": ([], None),
    "FreeCArray": ([c_void_p], None),
    "DeletePlaintext": ([c_int], None),
    "DeleteCiphertext": ([c_int], None),
    "GetPlaintextScale": ([c_int], c_ulong),
    "GetCiphertextScale": ([c_int], c_ulong),
    "SetPlaintextScale": ([c_int, c_ulong], None),
    "SetCiphertextScale": ([c_int, c_ulong], None),
    "GetPlaintextLevel": ([c_int], c_int),
    "GetCiphertextLevel": ([c_int], c_int),
    "GetPlaintextSlots": ([c_int], c_int),
    "GetCiphertextSlots": ([c_int], c_int),
    "GetCiphertextDegree": ([c_int], c_int),
    "GetModuliChain": ([], ArrayResultUInt64),
    "GetLivePlaintexts": ([], ArrayResultInt),
    "GetLiveCiphertexts": ([], ArrayResultInt),
    "CloneCiphertext": ([c_int], c_int),
    "NewKeyGenerator": ([], None),
    "GenerateSecretKey": ([], None),
    "GeneratePublicKey": ([], None),
    "GenerateRelinearizationKey": ([], None),
    "GenerateEvaluationKeys": ([], None),
    "SerializeSecretKey": ([], ArrayResultByte),
    "LoadSecretKey": ([P(ctypes.c_ubyte), c_ulong], None),
    "NewEncoder": ([], None),
    "Encode": ([P(c_float), c_int, c_int, c_ulong], c_int),
    "Decode": ([c_int], ArrayResultFloat),
    "NewEncryptor": ([], None),
    "NewDecryptor": ([], None),
    "Encrypt": ([c_int], c_int),
    "Decrypt": ([c_int], c_int),
    "NewEvaluator": ([], None),
    "AddRotationKey": ([c_int], None),
    "Negate": ([c_int], c_int),
    "Rotate": ([c_int, c_int], c_int),
    "RotateNew": ([c_int, c_int], c_int),
    "OrionHipRotateAdd": ([c_int, c_int], c_int),
    "Rescale": ([c_int], c_int),
    "RescaleNew": ([c_int], c_int),
    "AddScalar": ([c_int, c_float], c_int),
    "AddScalarNew": ([c_int, c_float], c_int),
    "SubScalar": ([c_int, c_float], c_int),
    "SubScalarNew": ([c_int, c_float], c_int),
    "MulScalarInt": ([c_int, c_int], c_int),
    "MulScalarIntNew": ([c_int, c_int], c_int),
    "MulScalarFloat": ([c_int, c_float], c_int),
    "MulScalarFloatNew": ([c_int, c_float], c_int),
    "AddPlaintext": ([c_int, c_int], c_int),
    "AddPlaintextNew": ([c_int, c_int], c_int),
    "SubPlaintext": ([c_int, c_int], c_int),
    "SubPlaintextNew": ([c_int, c_int], c_int),
    "MulPlaintext": ([c_int, c_int], c_int),
    "MulPlaintextNew": ([c_int, c_int], c_int),
    "AddCiphertext": ([c_int, c_int], c_int),
    "AddCiphertextNew": ([c_int, c_int], c_int),
    "SubCiphertext": ([c_int, c_int], c_int),
    "SubCiphertextNew": ([c_int, c_int], c_int),
    "MulRelinCiphertext": ([c_int, c_int], c_int),
    "MulRelinCiphertextNew": ([c_int, c_int], c_int),
    "NewPolynomialEvaluator": ([], None),
    "GenerateMonomial": ([P(c_float), c_int], c_int),
    "GenerateChebyshev": ([P(c_float), c_int], c_int),
    "EvaluatePolynomial": ([c_int, c_int, c_ulong], c_int),
    "GenerateMinimaxSignCoeffs": ([P(c_int), c_int, c_int, c_int, c_int, c_int], ArrayResultDouble),
    "NewLinearTransformEvaluator": ([], None),
    "GenerateLinearTransform": ([P(c_int), c_int, P(c_float), c_int, c_int, c_float, c_char_p], c_int),
    "EvaluateLinearTransform": ([c_int, c_int], c_int),
    "DeleteLinearTransform": ([c_int], None),
    "GetLinearTransformRotationKeys": ([c_int], ArrayResultInt),
    "GenerateLinearTransformRotationKey": ([c_int], None),
    "GenerateConsolidatedRotationKeys": ([P(c_int), c_int], None),
    "GenerateAndSerializeRotationKey": ([c_int], ArrayResultByte),
    "LoadRotationKey": ([P(ctypes.c_ubyte), c_ulong, c_ulong], None),
    "SerializeDiagonal": ([c_int, c_int], ArrayResultByte),
    "LoadPlaintextDiagonal": ([P(ctypes.c_ubyte), c_ulong, c_int, c_ulong], None),
    "RemovePlaintextDiagonals": ([c_int], None),
    "RemoveRotationKeys": ([], None),
    "ModDropCiphertext": ([c_int], c_int),
    "GetPolyDepth": ([c_int], c_int),
    "NewBootstrapper": ([P(c_int), c_int, c_int], None),
    "Bootstrap": ([c_int, c_int], c_int),
    "DeleteBootstrappers": ([], None),
    # ---- MI355X extensions ----
    "OrionHipLastError": ([], c_char_p),
    "OrionHipClearError": ([], None),
    "OrionHipSetDevice": ([c_int], c_int),
    "OrionHipSetSeed": ([c_ulong], None),
    "OrionHipSetStream": ([c_void_p], None),
    "OrionHipGetStream": ([], c_void_p),
    "OrionHipThreadPipelines": ([c_int], c_int),
    "OrionHipCurrentPipeline": ([], c_int),
    "OrionHipPoolCap": ([c_double], c_double),
    "OrionHipPeerCreate": ([], c_int),
    "OrionHipPeerSelect": ([c_int], c_int),
    "OrionHipPeerCount": ([], c_int),
    "OrionHipStreamWaitPeer": ([c_int], c_int),
    "OrionHipPoolStats": ([P(c_double), c_int], c_int),
    "OrionHipSynchronize": ([], c_int),
    "OrionHipGraphBegin": ([], c_int),
    "OrionHipGraphEnd": ([], c_int),
    "OrionHipGraphLaunch": ([c_int], c_int),
    "OrionHipGraphDestroy": ([c_int], None),
    "OrionHipLogN": ([], c_int),
    "OrionHipNumQ": ([], c_int),
    "OrionHipNumP": ([], c_int),
    "OrionHipModulus": ([c_int], c_ulong),
    "OrionHipBootstrapNumQ": ([c_int], c_int),
    "OrionHipBootstrapNumP": ([c_int], c_int),
    "OrionHipBootstrapModulus": ([c_int, c_int], c_ulong),
    "OrionHipBootstrapExport": ([c_int, c_int, ctypes.c_long, c_void_p, c_ulong], ctypes.c_long),
    "EncodeBatch": ([P(c_float), c_int, c_int, c_int, c_ulong], c_int),
    "EncodeBatchDevice": ([c_void_p, c_int, c_int, c_int, c_double], c_int),
    "DecodeDevice": ([c_int, c_void_p], c_int),
    "DecodeF64": ([c_int, P(c_double), c_ulong], c_int),
    "OrionHipEncryptionIndex": ([], ctypes.c_uint),
    "GetCiphertextBatch": ([c_int], c_int),
    "GetPlaintextBatch": ([c_int], c_int),
    "GetCiphertextScaleF": ([c_int], c_double),
    "ImportCiphertext": ([P(c_ulong), c_int, c_int, c_double], c_int),
    "ExportCiphertext": ([c_int, P(c_ulong), c_ulong], c_int),
    "ImportPlaintext": ([P(c_ulong), c_int, c_int, c_double], c_int),
    "ExportPlaintext": ([c_int, P(c_ulong), c_ulong], c_int),
    "ImportCiphertextDevice": ([c_void_p, c_int, c_int, c_double], c_int),
    "ExportCiphertextDevice": ([c_int, c_void_p, c_ulong], c_int),
    "ExportSecretKey": ([P(c_ulong), c_ulong], c_int),
    "ExportPublicKey": ([P(c_ulong), c_ulong], c_int),
    "ExportRelinKey": ([P(c_ulong), c_ulong], c_int),
    "ExportGaloisKey": ([c_ulong, P(c_ulong), c_ulong], c_int),
    "GetGaloisKeyLevel": ([c_ulong], c_int),
    "ExportLinearTransformDiagonal": ([c_int, c_int, P(c_ulong), c_ulong], c_int),
    "GetLinearTransformN1": ([c_int], c_int),
    "GaloisElement": ([c_int], c_ulong),
    "KeyBundleBytes": ([c_int], c_ulong),
    "ExportKeyBundle": ([c_void_p, c_int], c_int),
    "ImportKeyBundle": ([c_void_p, c_ulong], c_int),
    "OrionHipProfile": ([c_int], None),
    "OrionHipProfileRead": ([c_char_p, P(ctypes.c_long), P(c_double), P(c_double), c_int], c_int),
    "OrionHipProfileReadStrict": ([P(c_double), c_int], c_int),
    "OrionHipProfileReset": ([], None),
    "OrionHipProfileClock": ([], None),
    "OrionHipLogMark": ([c_char_p], None),
    "OrionHipProfileUnion": ([ctypes.c_uint], c_double),
    "OrionHipNTT": ([P(c_ulong), c_int, c_int, P(c_int), c_int], c_int),
}

# the symbols a binding of the reference's Lattigo backend resolves (bindings.py:141-746 + fork extras)
LATTIGO_SYMBOLS = [n for n in SIGNATURES if not n.startswith("OrionHip") and n not in (
    "EncodeBatch", "EncodeBatchDevice", "DecodeDevice", "DecodeF64", "GetCiphertextBatch", "GetPlaintextBatch",
    "GetCiphertextScaleF", "ImportCiphertext", "ExportCiphertext", "ImportPlaintext", "ExportPlaintext",
    "ImportCiphertextDevice", "ExportCiphertextDevice",
    "ExportSecretKey", "ExportPublicKey", "ExportRelinKey",
    "ExportGaloisKey", "GetGaloisKeyLevel", "ExportLinearTransformDiagonal", "GetLinearTransformN1", "GaloisElement",
    "KeyBundleBytes", "ExportKeyBundle", "ImportKeyBundle", "ModDropCiphertext", "GetPolyDepth")]


def _hip_runtimes():
    """Paths of the HIP runtime libraries mapped into this process."""
    with open("/proc/self/maps") as f:
        return sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})


def load_library(path=LIB_PATH):
    """Load liborion_hip.so and declare every symbol; raises if missing.

    torch is imported first, so that the process holds ONE HIP runtime: the
    torch wheel bundles its own libamdhip64 / libhsa-runtime64 and links them
    by the unversioned name (NEEDED libamdhip64.so), which does not match the
    versioned soname this library links (libamdhip64.so.7 from /opt/rocm).
    Loaded after this library, torch would map a second HIP and HSA runtime
    beside ours; under rocprofv3's HIP API interception a torch kernel launch
    was then routed into the other runtime and crashed (the r03p
    SIGSEGV).  Loaded after torch, this library binds to torch's runtime."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"HIP backend library not found at {path}: build it with "
            "`python orion_amd/build.py` (no CPU fallback exists)")
    try:
        import torch  # noqa: F401  (one HIP runtime per process; see above)
    except ImportError:  # no torch: this library's own runtime is the only one
        pass
    lib = ctypes.CDLL(path)
    rt = _hip_runtimes()
    if len(rt) > 1:
        raise RuntimeError(f"two HIP runtimes are mapped ({rt}): load torch before liborion_hip.so")
    for name, (args, res) in SIGNATURES.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    return lib


class HipFunction:
    """Mirror of LattigoFunction (bindings.py:10-66): converts Python lists to
    C arrays (floats -> C float), ArrayResult structs to lists (freed with
    FreeCArray), and raises on library errors."""

    def __init__(self, lib, name):
        self.lib = lib
        self.name = name
        self.func = getattr(lib, name)
        self.argtypes = self.func.argtypes or []

    def _convert(self, arg, typ):
        if isinstance(arg, bool):
            arg = int(arg)
        if isinstance(arg, (int, np.integer)) and typ in (c_int, c_ulong, c_float):
            return typ(float(arg)) if typ is c_float else typ(int(arg))
        if isinstance(arg, (float, np.floating)):
            return c_float(float(arg)) if typ is c_float else typ(arg)
        if isinstance(arg, str):
            return arg.encode("utf-8")
        if isinstance(arg, np.ndarray) and arg.dtype == np.uint8:
            arg = np.ascontiguousarray(arg)
            return (arg.ctypes.data_as(P(ctypes.c_ubyte)), len(arg))
        if isinstance(arg, (list, tuple, np.ndarray)):
            if typ == P(c_int):
                return ((c_int * len(arg))(*[int(x) for x in arg]), len(arg))
            if typ == P(c_float):
                a = np.ascontiguousarray(arg, dtype=np.float32)
                return (a.ctypes.data_as(P(c_float)), len(a), a)
            if typ == P(c_ulong):
                return ((c_ulong * len(arg))(*[int(x) for x in arg]), len(arg))
            raise ValueError(f"{self.name}: unexpected list argument for {typ}")
        return arg

    def __call__(self, *args):
        c_args, keep = [], []
        for arg in args:
            if len(c_args) >= len(self.argtypes) and keep and isinstance(arg, (int, np.integer)) \
                    and int(arg) == keep[-1][1]:
                # a list argument already supplied its length (LattigoFunction
                # expands a list to (ptr, len)); orion's poly_evaluator.py:23
                # passes len(coeffs) once more -- drop the duplicate
                continue
            typ = self.argtypes[len(c_args)] if len(c_args) < len(self.argtypes) else None
            c = self._convert(arg, typ)
            if isinstance(c, tuple):
                c_args.extend(c[:2])
                keep.append(c)
            else:
                c_args.append(c)
        self.lib.OrionHipClearError()
        res = self.func(*c_args)
        err = self.lib.OrionHipLastError()
        if err:
            raise RuntimeError(f"{self.name}: {err.decode()}")
        if isinstance(res, (ArrayResultFloat, ArrayResultDouble)):
            out = [float(res.Data[i]) for i in range(res.Length)]
            self.lib.FreeCArray(ctypes.cast(res.Data, c_void_p))
            return out
        if isinstance(res, (ArrayResultInt, ArrayResultUInt64)):
            out = [int(res.Data[i]) for i in range(res.Length)]
            self.lib.FreeCArray(ctypes.cast(res.Data, c_void_p))
            return out
        if isinstance(res, ArrayResultByte):
            buf = ctypes.cast(res.Data, P(ctypes.c_ubyte * res.Length)).contents if res.Length else b""
            arr = np.frombuffer(bytes(buf), dtype=np.uint8).copy()
            self.lib.FreeCArray(ctypes.cast(res.Data, c_void_p))
            return arr, None
        return res


# The scheme is process-global, like Lattigo's (scheme.go:32): every
# HipLibrary of a process drives the same one.  A generation number, bumped by
# each NewScheme / DeleteScheme, lets a holder tell whether the scheme it set
# up is still the live one (scheme_current).
_SCHEME_GEN = [0]


class HipLibrary:
    """Drop-in replacement for LattigoLibrary (bindings.py:94-139)."""

    def __init__(self, path=LIB_PATH):
        self.lib = load_library(path)
        for name in SIGNATURES:
            setattr(self, name, HipFunction(self.lib, name))
        self._scheme_gen = None
        new, delete = self.NewScheme, self.DeleteScheme

        def new_scheme_call(*args):
            _SCHEME_GEN[0] += 1
            self._scheme_gen = None
            new(*args)
            self._scheme_gen = _SCHEME_GEN[0]

        def delete_scheme_call(*args):
            _SCHEME_GEN[0] += 1
            delete(*args)

        self.NewScheme, self.DeleteScheme = new_scheme_call, delete_scheme_call

    def scheme_current(self):
        """True while the scheme this object created is the process's live one."""
        return self._scheme_gen is not None and self._scheme_gen == _SCHEME_GEN[0]

    # evaluator.py:30-41 calls the HEonGPU binding's private
    # _ModDropCiphertext(arithmeticoperator_handle, ct, None)
    arithmeticoperator_handle = None

    def _ModDropCiphertext(self, handle, ct, _stream=None):
        return self.ModDropCiphertext(ct)

    def setup_bindings(self, orion_params):
        """Same flow as LattigoLibrary.setup_bindings -> NewScheme (bindings.py:126-179)."""
        self.NewScheme(
            orion_params.get_logn(), orion_params.get_logq(), orion_params.get_logp(),
            orion_params.get_logscale(), orion_params.get_hamming_weight(), orion_params.get_ringtype(),
            orion_params.get_keys_path(), orion_params.get_io_mode())

    # ---- numpy helpers for tests / bench (extension API) ----------------
    def new_scheme(self, logn, logq, logp, logscale=None, h=192, ringtype="standard", seed=None, device=None):
        if device is not None:
            if self.OrionHipSetDevice(device) != 0:
                raise RuntimeError("OrionHipSetDevice failed")
        if seed is not None:
            self.OrionHipSetSeed(seed)
        self.NewScheme(logn, list(logq), list(logp), logscale or logq[-1], h, ringtype, "", "none")
        self.N = 1 << self.OrionHipLogN()  # coefficients per limb (both rings)
        ci = str(ringtype).lower() != "standard"
        self.slots = self.N if ci else self.N // 2  # ConjugateInvariant: N real slots (scheme.go:49-52)
        self.L, self.K = len(logq), len(logp)
        return self

    def moduli(self):
        return [int(self.OrionHipModulus(i)) for i in range(self.L + self.K)]

    def bootstrap_moduli(self, slots):
        """(Q primes, P primes) of the bootstrapping chain of the circuit for `slots`."""
        nq, npr = self.OrionHipBootstrapNumQ(slots), self.OrionHipBootstrapNumP(slots)
        if nq < 0:
            raise RuntimeError(f"no bootstrapper found for slot count: {slots}")
        m = [int(self.OrionHipBootstrapModulus(slots, i)) for i in range(nq + npr)]
        return m[:nq], m[nq:]

    BTX = dict(params=0, cos=1, trace=2, rlk=3, galois_keys=4, galois=5, lt_info=6, lt_diag=7, mono_i=8,
               d2s=9, s2d=10)

    def bootstrap_export(self, slots, what, arg=0):
        """A bootstrapper's keys (the CPU oracle's only shared inputs) and, for
        comparison with the oracle's own derivation, its constants and diagonals
        (OrionHipBootstrapExport)."""
        w = self.BTX[what]
        n = self._chk(self.lib.OrionHipBootstrapExport(slots, w, arg, None, 0), "OrionHipBootstrapExport")
        dt = {0: np.longdouble, 1: np.longdouble, 6: np.int64}.get(w, np.uint64)
        out = np.zeros(n, dtype=dt)
        self._chk(self.lib.OrionHipBootstrapExport(slots, w, arg, out.ctypes.data_as(c_void_p), n),
                  "OrionHipBootstrapExport")
        return out

    def thread_pipelines(self, n):
        """Thread-affine pipelines (OrionHipThreadPipelines): with n > 1 every
        thread other than the scheme's gets a context of its own at its first
        call -- the scheme's keys and compiled objects, its own stream, pool
        and handles -- so threads each running the frontend's forward pass
        overlap on the GPU.  Returns the previous setting."""
        return int(self.lib.OrionHipThreadPipelines(int(n)))

    def pool_cap(self, nbytes):
        """Cap on the device bytes all pools hold (0: none); returns the previous cap."""
        return float(self.lib.OrionHipPoolCap(float(nbytes)))

    def pool_stats(self):
        """Device-memory pools (OrionHipPoolStats): bytes held and their peak,
        hipMalloc calls, failed allocations that forced a trim of every cache,
        bytes cached."""
        v = (c_double * 5)()
        self.lib.OrionHipPoolStats(v, 5)
        return {"held_bytes": v[0], "peak_bytes": v[1], "hipmalloc_calls": int(v[2]), "trims": int(v[3]),
                "cached_bytes": v[4]}

    def export_ciphertext(self, ct):
        B, lvl = self.GetCiphertextBatch(ct), self.GetCiphertextLevel(ct)
        out = np.zeros((B, 2, lvl + 1, self.N), dtype=np.uint64)
        self._chk(self.lib.ExportCiphertext(ct, out.ctypes.data_as(P(c_ulong)), out.size), "ExportCiphertext")
        return out

    def import_ciphertext(self, arr, scale):
        arr = np.ascontiguousarray(arr, dtype=np.uint64)
        if arr.ndim == 3:
            arr = arr[None]
        B, _, nl, _ = arr.shape
        h = self.lib.ImportCiphertext(arr.ctypes.data_as(P(c_ulong)), B, nl - 1, float(scale))
        return self._chk(h, "ImportCiphertext")

    # Device-pointer calls run asynchronously on the library stream, which
    # torch does not know about: order them against the tensor's stream both
    # ways, and keep an input tensor from being recycled by torch's caching
    # allocator before the copy that reads it has run.
    def _streams(self, t):
        import torch
        cur = torch.cuda.current_stream(t.device)
        ptr = self.OrionHipGetStream()
        lib_s = torch.cuda.ExternalStream(ptr, device=t.device) if ptr else torch.cuda.default_stream(t.device)
        return cur, lib_s

    def _before_read(self, t):
        cur, lib_s = self._streams(t)
        lib_s.wait_stream(cur)  # the producer of t runs first
        return lib_s

    def _before_write(self, t):
        cur, lib_s = self._streams(t)
        lib_s.wait_stream(cur)  # earlier torch work on t (allocation, readers) first
        return cur, lib_s

    def import_ciphertext_device(self, t, scale):
        """t: a contiguous [B][2][level+1][N] int64/uint64 device tensor (torch),
        NTT domain, every residue fully reduced."""
        assert t.is_cuda and t.is_contiguous() and t.dim() == 4 and t.shape[3] == self.N and t.element_size() == 8
        lib_s = self._before_read(t)
        h = self._chk(self.lib.ImportCiphertextDevice(t.data_ptr(), t.shape[0], t.shape[2] - 1, float(scale)),
                      "ImportCiphertextDevice")
        t.record_stream(lib_s)
        return h

    def export_ciphertext_device(self, ct, out):
        """Copy ciphertext `ct` into the device tensor `out` ([B][2][level+1][N], 8-byte elements)."""
        assert out.is_cuda and out.is_contiguous() and out.element_size() == 8
        cur, lib_s = self._before_write(out)
        self._chk(self.lib.ExportCiphertextDevice(ct, out.data_ptr(), out.numel()), "ExportCiphertextDevice")
        cur.wait_stream(lib_s)  # torch's readers of out follow the copy
        return out

    def decode_device(self, pt, out):
        """Real parts of every slot of every image into the float64 device tensor out [B][slots]."""
        assert out.is_cuda and out.is_contiguous() and out.dtype.itemsize == 8
        cur, lib_s = self._before_write(out)
        self._chk(self.lib.DecodeDevice(pt, out.data_ptr()), "DecodeDevice")
        cur.wait_stream(lib_s)
        return out

    def export_plaintext(self, pt):
        B = self.GetPlaintextBatch(pt)
        lvl = self.GetPlaintextLevel(pt)
        out = np.zeros((B, lvl + 1, self.N), dtype=np.uint64)
        self._chk(self.lib.ExportPlaintext(pt, out.ctypes.data_as(P(c_ulong)), out.size), "ExportPlaintext")
        return out

    def import_plaintext(self, arr, scale):
        arr = np.ascontiguousarray(arr, dtype=np.uint64)
        if arr.ndim == 2:
            arr = arr[None]
        B, nl, _ = arr.shape
        return self._chk(self.lib.ImportPlaintext(arr.ctypes.data_as(P(c_ulong)), B, nl - 1, float(scale)),
                         "ImportPlaintext")

    def export_secret_key(self):
        out = np.zeros((self.L + self.K, self.N), dtype=np.uint64)
        self._chk(self.lib.ExportSecretKey(out.ctypes.data_as(P(c_ulong)), out.size), "ExportSecretKey")
        return out

    def export_public_key(self):
        out = np.zeros((2, self.L + self.K, self.N), dtype=np.uint64)
        self._chk(self.lib.ExportPublicKey(out.ctypes.data_as(P(c_ulong)), out.size), "ExportPublicKey")
        return out

    def _evk_shape(self):
        return ((self.L + self.K - 1) // self.K, 2, self.L + self.K, self.N)

    def export_relin_key(self):
        out = np.zeros(self._evk_shape(), dtype=np.uint64)
        self._chk(self.lib.ExportRelinKey(out.ctypes.data_as(P(c_ulong)), out.size), "ExportRelinKey")
        return out

    def export_galois_key(self, galEl):
        out = np.zeros(self._evk_shape(), dtype=np.uint64)
        self._chk(self.lib.ExportGaloisKey(galEl, out.ctypes.data_as(P(c_ulong)), out.size), "ExportGaloisKey")
        return out

    def export_lt_diagonal(self, lt, idx, level):
        out = np.zeros((level + 1 + self.K, self.N), dtype=np.uint64)
        self._chk(self.lib.ExportLinearTransformDiagonal(lt, idx, out.ctypes.data_as(P(c_ulong)), out.size),
                  "ExportLinearTransformDiagonal")
        return out

    def encode_batch(self, values, level, scale):
        v = np.ascontiguousarray(values, dtype=np.float32)
        B, n = v.shape
        return self._chk(self.lib.EncodeBatch(v.ctypes.data_as(P(c_float)), n, B, level, int(scale)), "EncodeBatch")

    def encode_batch_device(self, dvalues, level, scale):
        """dvalues: a contiguous float32 [B][n] device tensor (torch, HBM resident)."""
        B, n = dvalues.shape
        lib_s = self._before_read(dvalues)
        h = self._chk(self.lib.EncodeBatchDevice(dvalues.data_ptr(), n, B, level, float(scale)),
                      "EncodeBatchDevice")
        dvalues.record_stream(lib_s)
        return h

    def decode_f64(self, pt):
        """Slots of every image of a plaintext, float64 [B][slots] (GPU decode)."""
        out = np.zeros((self.GetPlaintextBatch(pt), self.GetPlaintextSlots(pt)), dtype=np.float64)
        self._chk(self.lib.DecodeF64(pt, out.ctypes.data_as(P(c_double)), out.size), "DecodeF64")
        return out

    def profile_read(self):
        n = 16
        names = ctypes.create_string_buffer(32 * n)
        launches = (ctypes.c_long * n)()
        ms = (c_double * n)()
        byts = (c_double * n)()
        strict = (c_double * n)()
        k = self.lib.OrionHipProfileRead(names, launches, ms, byts, n)
        self.lib.OrionHipProfileReadStrict(strict, n)
        out = {}
        for i in range(max(k, 0)):
            nm = names.raw[32 * i:32 * i + 32].split(b"\0")[0].decode()
            out[nm] = dict(launches=int(launches[i]), ms=float(ms[i]), bytes=float(byts[i]),
                           strict_bytes=float(strict[i]))
        return out

    def profile_union(self, mask):
        """ms of wall clock with at least one profiled launch of a category in
        `mask` running, over every context, since OrionHipProfileClock."""
        v = self.lib.OrionHipProfileUnion(mask)
        if v < 0:
            raise RuntimeError(f"OrionHipProfileUnion: {self.lib.OrionHipLastError().decode()}")
        return v

    def _chk(self, rc, name):
        if rc is None or (isinstance(rc, int) and rc < 0):
            raise RuntimeError(f"{name}: {self.lib.OrionHipLastError().decode()}")
        return rc
