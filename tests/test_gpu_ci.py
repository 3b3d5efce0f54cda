"""GPU parity tests of the native ConjugateInvariant ring (scheme.go:49-52:
Z[X + X^-1]/(X^2N + 1) of degree N, NthRoot 4N, N real slots) vs the oracle's
CI ring (oracle_new_ring, pinned to the degree-2N Standard ring in
tests/test_oracle.py).  N coefficients per limb; the forward NTT folds its
input and the inverse unfolds its output inside the one-pass kernels
(ntt.hip).  Integer ring arithmetic must match bit for bit."""
import ctypes

import numpy as np
import pytest

from tests.helpers import rand_ct, SchemeCache

pytestmark = pytest.mark.gpu

CI_SMALL = dict(logn=13, logq=[55, 40, 40, 40, 40, 40], logp=[60, 60])


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


_ci_small_cache = SchemeCache()


@pytest.fixture
def ci_small(torch_cuda, oracle_mod):
    """function-scoped view of a module-wide scheme, rebuilt if another test
    replaced the process-global scheme (order-independent)"""

    def make():
        from orion_amd.backend import HipLibrary
        p = CI_SMALL
        lib = HipLibrary().new_scheme(p["logn"], p["logq"], p["logp"], 40, h=192, seed=4321,
                                      ringtype="ConjugateInvariant")
        mods = lib.moduli()
        assert mods == oracle_mod.gen_moduli(p["logn"] + 1, p["logq"], p["logp"])  # q = 1 mod 4N
        orc = oracle_mod.Oracle(p["logn"], mods, len(p["logq"]), len(p["logp"]), ci=True)
        assert lib.N == orc.N == 1 << p["logn"] and lib.slots == orc.slots == orc.N
        lib.GenerateSecretKey()
        lib.GeneratePublicKey()
        lib.GenerateRelinearizationKey()
        return lib, orc

    return _ci_small_cache.get(make)


def _ntt_roundtrip(torch, lib, orc, host):
    """host: [limb][B][N] residues; forward on the GPU vs the oracle, then back."""
    nl, B = host.shape[0], host.shape[1]
    dev = torch.from_numpy(host.view(np.int64).copy()).cuda()
    mods_c = (ctypes.c_int * nl)(*range(nl))
    ptr = ctypes.cast(dev.data_ptr(), ctypes.POINTER(ctypes.c_ulong))
    assert lib.lib.OrionHipNTT(ptr, nl, B, mods_c, 0) == 0
    lib.OrionHipSynchronize()
    fwd = dev.cpu().numpy().view(np.uint64).copy()
    for m in range(nl):
        for b in range(B):
            assert np.array_equal(fwd[m, b], orc.ntt(m, host[m, b])), (m, b)
    assert lib.lib.OrionHipNTT(ptr, nl, B, mods_c, 1) == 0
    lib.OrionHipSynchronize()
    assert np.array_equal(dev.cpu().numpy().view(np.uint64), host)
    return fwd


@pytest.mark.parametrize("logn", [13, 14, 15])
def test_ci_ntt_parity(torch_cuda, oracle_mod, logn):
    """CI NTT/INTT on a 60/40/29/26-bit chain (integer path, reduced and lazy
    float64 paths), random limbs plus edge rows (0, 1, q-1, a lone X^0, a lone
    X^(N/2): the fold's self-paired coefficients)."""
    from orion_amd.backend import HipLibrary
    logq, logp = [60, 40, 29, 26], [60, 45]
    lib = HipLibrary().new_scheme(logn, logq, logp, 26, ringtype="ConjugateInvariant")
    mods = lib.moduli()
    orc = oracle_mod.Oracle(logn, mods, len(logq), len(logp), ci=True)
    N, nl = 1 << logn, len(mods)
    rng = np.random.default_rng(logn + 7)
    B = 7
    host = np.stack([rng.integers(0, mods[m], (B, N), dtype=np.uint64) for m in range(nl)])
    for m in range(nl):
        host[m, 1] = 0
        host[m, 2] = 1
        host[m, 3] = mods[m] - 1
        host[m, 4] = 0
        host[m, 4, 0] = mods[m] - 1
        host[m, 5] = 0
        host[m, 5, N // 2] = 12345
    fwd = _ntt_roundtrip(torch_cuda, lib, orc, host)
    assert not fwd[:, 1].any()
    lib.DeleteScheme()


def test_ci_ntt_persistent_batch(torch_cuda, oracle_mod):
    """More limb-transforms than workgroups (6 limbs x 48 = 288 > 256 CUs): the
    persistent kernels walk several jobs per workgroup through the unfold's
    LDS staging."""
    from orion_amd.backend import HipLibrary
    logq, logp = [60, 40, 40, 40], [60, 60]
    lib = HipLibrary().new_scheme(13, logq, logp, 40, ringtype="ConjugateInvariant")
    mods = lib.moduli()
    orc = oracle_mod.Oracle(13, mods, len(logq), len(logp), ci=True)
    rng = np.random.default_rng(99)
    host = np.stack([rng.integers(0, mods[m], (48, 1 << 13), dtype=np.uint64) for m in range(len(mods))])
    _ntt_roundtrip(torch_cuda, lib, orc, host)
    lib.DeleteScheme()


def test_ci_encode_decode_parity(ci_small):
    """GPU encode (N real slots: special iFFT of size N, real parts only) and
    decode (slot j = a_j - i a_{N-j}) bit for bit vs the oracle."""
    lib, orc = ci_small
    rng = np.random.default_rng(21)
    level, B = 3, 2
    vals = rng.uniform(-3, 3, (B, orc.slots - 9)).astype(np.float32)
    got = lib.export_plaintext(lib.encode_batch(vals, level, 1 << 40))
    for b in range(B):
        assert np.array_equal(got[b], orc.encode(vals[b].astype(np.float64), 2.0 ** 40, list(range(level + 1)))), b
    dp = lib.Decrypt(lib.Encrypt(lib.encode_batch(vals, level, 1 << 40)))
    dec = lib.decode_f64(dp)
    raw = lib.export_plaintext(dp)
    assert dec.shape == (B, orc.slots)
    for b in range(B):
        assert np.array_equal(dec[b], orc.decode(raw[b], level, 2.0 ** 40)), b
        assert np.abs(dec[b, :vals.shape[1]] - vals[b]).max() < 1e-4
        assert np.abs(dec[b, vals.shape[1]:]).max() < 1e-4


def test_ci_encrypt_parity(ci_small):
    lib, orc = ci_small
    rng = np.random.default_rng(22)
    level, B = 4, 2
    vals = rng.uniform(-1, 1, (B, orc.slots)).astype(np.float32)
    pt = lib.encode_batch(vals, level, 1 << 40)
    ptv = lib.export_plaintext(pt)
    pk = lib.export_public_key()
    enc = int(lib.OrionHipEncryptionIndex())
    got = lib.export_ciphertext(lib.Encrypt(pt))
    for b in range(B):
        assert np.array_equal(got[b], orc.encrypt_pk(4321, enc, b, pk, ptv[b], level)), b


def test_ci_mul_relin_rescale_parity(ci_small):
    lib, orc = ci_small
    rng = np.random.default_rng(23)
    level = 5
    a = rand_ct(rng, orc.moduli, level, orc.N, B=2)
    b = rand_ct(rng, orc.moduli, level, orc.N, B=2)
    cc = lib.MulRelinCiphertextNew(lib.import_ciphertext(a, 2.0 ** 40), lib.import_ciphertext(b, 2.0 ** 40))
    rlk = lib.export_relin_key()
    ref = [orc.mul_relin(a[i], b[i], rlk, level) for i in range(2)]
    got = lib.export_ciphertext(cc)
    for i in range(2):
        assert np.array_equal(got[i], ref[i]), i
    for lv in range(level, 0, -1):
        lib.Rescale(cc)
        got = lib.export_ciphertext(cc)
        for i in range(2):
            ref[i] = orc.rescale(ref[i], lv)
            assert np.array_equal(got[i], ref[i]), (lv, i)


def test_ci_rotate_parity(ci_small):
    """Galois elements 5^k mod 4N; rotations are cyclic over the N real slots."""
    lib, orc = ci_small
    rng = np.random.default_rng(24)
    level = 3
    a = rand_ct(rng, orc.moduli, level, orc.N, B=1)
    ca = lib.import_ciphertext(a, 2.0 ** 40)
    for k in [1, 5, -3, 1000, orc.slots - 1]:
        g = int(lib.GaloisElement(k))
        assert g == orc.galois_element(k) == pow(5, k % (4 * orc.N), 4 * orc.N)
        cr = lib.RotateNew(ca, k)
        got = lib.export_ciphertext(cr)[0]
        assert np.array_equal(got, orc.rotate(a[0], g, lib.export_galois_key(g), level)), k
    vals = rng.standard_normal(orc.slots).astype(np.float32)
    ct = lib.Encrypt(lib.Encode(list(vals), 5, 1 << 40))
    dec = np.array(lib.Decode(lib.Decrypt(lib.RotateNew(ct, 7))))
    assert dec.shape == (orc.slots,)
    assert np.abs(dec - np.roll(vals, -7)).max() < 1e-3


def test_ci_linear_transform_parity(ci_small):
    lib, orc = ci_small
    rng = np.random.default_rng(25)
    slots, level = orc.slots, 4
    idx = [0, 1, 2, 3, 17, 64, 65, 300, 5000, slots - 1]
    diags = rng.uniform(-1, 1, (len(idx), slots)).astype(np.float32)
    lt = lib.GenerateLinearTransform(idx, list(diags.reshape(-1)), level, 2.0, "none")
    gels = lib.GetLinearTransformRotationKeys(lt)
    lib.GenerateConsolidatedRotationKeys(gels)
    vals = rng.standard_normal(slots).astype(np.float32)
    ct = lib.Encrypt(lib.Encode(list(vals), level, 1 << 40))
    x = lib.export_ciphertext(ct)[0]
    out = lib.EvaluateLinearTransform(lt, ct)
    N1 = lib.GetLinearTransformN1(lt)
    assert N1 == orc.find_best_bsgs_n1(idx, 0)
    pts = [lib.export_lt_diagonal(lt, d, level) for d in idx]
    gkeys = {g: lib.export_galois_key(g) for g in gels if g != 1}
    assert np.array_equal(lib.export_ciphertext(out)[0], orc.lt_bsgs(x, level, idx, pts, N1, gkeys))
    lib.Rescale(out)
    dec = np.array(lib.Decode(lib.Decrypt(out)))
    exp = sum(diags[i].astype(np.float64) * np.roll(vals, -d) for i, d in enumerate(idx))
    assert np.abs(dec - exp).max() < 1e-3


def test_ci_rejects_bootstrapping(ci_small):
    lib, _ = ci_small
    with pytest.raises(RuntimeError, match="Standard ring"):
        lib.NewBootstrapper([61], 1 << 12)
