"""CPU tests of the drop-in boundary: liborion_hip.so builds for gfx950, loads,
exports every symbol include/orion_hip.h declares (the Lattigo binding's
symbol set + the fork's extras), and fails loudly -- never falls back to a
CPU path -- when no GPU is present."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "orion_hip.h")
REF_BINDINGS_SYMBOLS = [
    # every self.lib.<name> the reference's LattigoLibrary binds (bindings.py:141-746)
    "NewScheme", "DeleteScheme", "FreeCArray", "DeletePlaintext", "DeleteCiphertext", "GetPlaintextScale",
    "GetCiphertextScale", "SetPlaintextScale", "SetCiphertextScale", "GetPlaintextLevel", "GetCiphertextLevel",
    "GetPlaintextSlots", "GetCiphertextSlots", "GetCiphertextDegree", "GetModuliChain", "GetLivePlaintexts",
    "GetLiveCiphertexts", "NewKeyGenerator", "GenerateSecretKey", "GeneratePublicKey",
    "GenerateRelinearizationKey", "GenerateEvaluationKeys", "SerializeSecretKey", "LoadSecretKey", "NewEncoder",
    "Encode", "Decode", "NewEncryptor", "NewDecryptor", "Encrypt", "Decrypt", "NewEvaluator", "AddRotationKey",
    "Negate", "Rotate", "RotateNew", "Rescale", "RescaleNew", "AddScalar", "AddScalarNew", "SubScalar",
    "SubScalarNew", "MulScalarInt", "MulScalarIntNew", "MulScalarFloat", "MulScalarFloatNew", "AddPlaintext",
    "AddPlaintextNew", "SubPlaintext", "SubPlaintextNew", "MulPlaintext", "MulPlaintextNew", "AddCiphertext",
    "AddCiphertextNew", "SubCiphertext", "SubCiphertextNew", "MulRelinCiphertext", "MulRelinCiphertextNew",
    "NewPolynomialEvaluator", "GenerateMonomial", "GenerateChebyshev", "EvaluatePolynomial",
    "GenerateMinimaxSignCoeffs", "NewLinearTransformEvaluator", "GenerateLinearTransform",
    "EvaluateLinearTransform", "DeleteLinearTransform", "GetLinearTransformRotationKeys",
    "GenerateLinearTransformRotationKey", "GenerateAndSerializeRotationKey", "LoadRotationKey",
    "SerializeDiagonal", "LoadPlaintextDiagonal", "RemovePlaintextDiagonals", "RemoveRotationKeys",
    "NewBootstrapper", "Bootstrap", "DeleteBootstrappers",
    # fork extras called by orion/backend/python (lt_evaluator.py:77, tensors.py:229)
    "GenerateConsolidatedRotationKeys", "CloneCiphertext",
]


@pytest.fixture(scope="module")
def libpath():
    from orion_amd import build
    return build.build()


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", txt)
    return sorted(set(n for n in names if n not in ("if", "while", "return", "sizeof")))


def test_library_is_gfx950(libpath):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", libpath], capture_output=True, text=True)
    blob = open(libpath, "rb").read()
    assert b"gfx950" in blob, "no gfx950 code object in liborion_hip.so"


def test_exports_every_header_symbol(libpath):
    import torch  # noqa: F401  (torch's HIP runtime first: one runtime per process, backend.load_library)
    lib = ctypes.CDLL(libpath)
    syms = header_symbols()
    assert len(syms) > 100
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_header_covers_reference_binding(libpath):
    syms = set(header_symbols())
    missing = [s for s in REF_BINDINGS_SYMBOLS if s not in syms]
    assert not missing, missing


def test_python_binding_declares_all(libpath):
    from orion_amd.backend import SIGNATURES, load_library
    load_library()
    assert set(REF_BINDINGS_SYMBOLS) <= set(SIGNATURES)
    assert set(SIGNATURES) <= set(header_symbols())


def test_no_cpu_fallback_without_gpu(libpath):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from orion_amd.backend import HipLibrary
    lib = HipLibrary()
    with pytest.raises(RuntimeError):
        lib.new_scheme(13, [50, 40], [60])


def test_missing_library_raises(tmp_path):
    from orion_amd.backend import load_library
    with pytest.raises(RuntimeError):
        load_library(str(tmp_path / "nope.so"))


def test_lattigo_style_conversions(libpath):
    """HipFunction mirrors LattigoFunction's argument conversions (bindings.py:40-66)."""
    from orion_amd.backend import HipFunction, load_library, ArrayResultInt
    lib = load_library()
    f = HipFunction(lib, "Encode")
    c = f._convert([1.0, 2.5], f.argtypes[0])
    assert c[1] == 2
    g = HipFunction(lib, "AddScalar")
    assert isinstance(g._convert(0.5, g.argtypes[1]), ctypes.c_float)
    h = HipFunction(lib, "GenerateConsolidatedRotationKeys")
    arr, n = h._convert([5, 25], h.argtypes[0])
    assert n == 2 and arr[1] == 25


def test_ring_type_contract(libpath):
    """scheme.go:50-51 accepts "standard" and (any other string as)
    ConjugateInvariant; this backend names the two it supports and rejects
    the rest, and a CI ring of degree 2^16 (its fold/unfold runs in the
    one-limb-per-CU NTT, N <= 2^15) with an error string instead of an abort.  Both checks run before any
    device call, so they hold on a CPU-only host."""
    from orion_amd.backend import HipLibrary
    lib = HipLibrary()
    with pytest.raises(RuntimeError, match="unknown ring type"):
        lib.NewScheme(13, [29, 26], [29], 26, 192, "Bogus", "", "none")
    with pytest.raises(RuntimeError, match="logN must be 13..15"):
        lib.NewScheme(16, [60, 40], [60], 40, 192, "ConjugateInvariant", "", "none")
