"""GPU parity tests: the HIP backend (through the C-ABI) vs the CPU oracle on
the same inputs.  Integer ring arithmetic must match bit for bit."""
import numpy as np
import pytest

from tests.helpers import SMALL, rand_ct, SchemeCache, bootstrap_keys, bootstrap_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


_small_cache = SchemeCache()


@pytest.fixture
def small(torch_cuda, oracle_mod):
    """function-scoped view of a module-wide scheme, rebuilt if another test
    replaced the process-global scheme (order-independent)"""

    def make():
        from orion_amd.backend import HipLibrary
        lib = HipLibrary().new_scheme(SMALL["logn"], SMALL["logq"], SMALL["logp"], 40, h=192, seed=1234)
        mods = lib.moduli()
        orc = oracle_mod.Oracle(SMALL["logn"], mods, len(SMALL["logq"]), len(SMALL["logp"]))
        lib.GenerateSecretKey()
        lib.GeneratePublicKey()
        lib.GenerateRelinearizationKey()
        return lib, orc

    return _small_cache.get(make)


@pytest.mark.parametrize("logn", [13, 14, 15, 16])
def test_ntt_roundtrip_and_parity(torch_cuda, oracle_mod, logn):
    torch = torch_cuda
    from orion_amd.backend import HipLibrary
    import ctypes
    logq = [60] + [40] * 3
    lib = HipLibrary().new_scheme(logn, logq, [60, 60], 40)
    mods = lib.moduli()
    assert mods == oracle_mod.gen_moduli(logn, logq, [60, 60])
    orc = oracle_mod.Oracle(logn, mods, len(logq), 2)
    N, B = 1 << logn, 3
    nl = len(mods)
    rng = np.random.default_rng(logn)
    host = np.stack([rng.integers(0, mods[m], (B, N), dtype=np.uint64) for m in range(nl)])  # [limb][b][N]
    dev = torch.from_numpy(host.view(np.int64).copy()).cuda()
    mods_c = (ctypes.c_int * nl)(*range(nl))
    ptr = ctypes.cast(dev.data_ptr(), ctypes.POINTER(ctypes.c_ulong))
    assert lib.lib.OrionHipNTT(ptr, nl, B, mods_c, 0) == 0
    lib.OrionHipSynchronize()
    fwd = dev.cpu().numpy().view(np.uint64)
    for m in range(nl):
        for b in range(B):
            assert np.array_equal(fwd[m, b], orc.ntt(m, host[m, b])), (m, b)
    assert lib.lib.OrionHipNTT(ptr, nl, B, mods_c, 1) == 0
    lib.OrionHipSynchronize()
    back = dev.cpu().numpy().view(np.uint64)
    assert np.array_equal(back, host)
    lib.DeleteScheme()


@pytest.mark.parametrize("B", [32, 64])
def test_ntt_one_pass_launches(torch_cuda, oracle_mod, B):
    """N = 2^15 launches of one or two full rounds of 256 limb-transforms take
    the one-limb-per-workgroup kernels (smaller or partial-round launches take
    the two-pass kernels): integer-path (60-bit) and float64-path (40-bit)
    limbs in one launch, forward bit-exact with the oracle, inverse exact."""
    torch = torch_cuda
    from orion_amd.backend import HipLibrary
    import ctypes
    logn, logq = 15, [60] + [40] * 5
    lib = HipLibrary().new_scheme(logn, logq, [60, 60], 40)
    mods = lib.moduli()
    orc = oracle_mod.Oracle(logn, mods, len(logq), 2)
    N, nl = 1 << logn, len(mods)
    assert nl * B in (256, 512)
    rng = np.random.default_rng(B)
    host = np.stack([rng.integers(0, mods[m], (B, N), dtype=np.uint64) for m in range(nl)])
    host[:, 0, :8] = np.array([mods[m] - 1 for m in range(nl)], dtype=np.uint64)[:, None]
    dev = torch.from_numpy(host.view(np.int64).copy()).cuda()
    mods_c = (ctypes.c_int * nl)(*range(nl))
    ptr = ctypes.cast(dev.data_ptr(), ctypes.POINTER(ctypes.c_ulong))
    assert lib.lib.OrionHipNTT(ptr, nl, B, mods_c, 0) == 0
    lib.OrionHipSynchronize()
    fwd = dev.cpu().numpy().view(np.uint64).copy()
    for m in range(nl):
        for b in (0, B - 1):
            assert np.array_equal(fwd[m, b], orc.ntt(m, host[m, b])), (m, b)
    assert lib.lib.OrionHipNTT(ptr, nl, B, mods_c, 1) == 0
    lib.OrionHipSynchronize()
    back = dev.cpu().numpy().view(np.uint64)
    bad = [(m, b) for m in range(nl) for b in range(B) if not np.array_equal(back[m, b], host[m, b])]
    assert not bad, bad[:8]
    # inverse on its own against the oracle (inputs: arbitrary NTT-domain rows)
    dev.copy_(torch.from_numpy(host.view(np.int64).copy()))
    assert lib.lib.OrionHipNTT(ptr, nl, B, mods_c, 1) == 0
    lib.OrionHipSynchronize()
    inv = dev.cpu().numpy().view(np.uint64)
    for m in range(nl):
        assert np.array_equal(inv[m, 0], orc.intt(m, host[m, 0])), m
    lib.DeleteScheme()


def test_encode_parity(small):
    lib, orc = small
    rng = np.random.default_rng(1)
    vals = rng.standard_normal(orc.N // 2).astype(np.float32)
    level = 4
    pt = lib.Encode(list(vals), level, 1 << 40)
    got = lib.export_plaintext(pt)[0]
    ref = orc.encode(vals.astype(np.float64), 2.0 ** 40, list(range(level + 1)))
    assert np.array_equal(got, ref)


def test_encrypt_decrypt(small):
    lib, orc = small
    rng = np.random.default_rng(2)
    vals = rng.standard_normal(orc.N // 2).astype(np.float32)
    pt = lib.Encode(list(vals), 5, 1 << 40)
    ct = lib.Encrypt(pt)
    dec = np.array(lib.Decode(lib.Decrypt(ct)))
    assert np.abs(dec - vals).max() < 1e-4


def test_encode_batch_and_device_parity(small, torch_cuda):
    """GPU encode (special iFFT + fixed-point CRT + NTT, encoder.hip) of B
    different ragged images, from host memory and from a device tensor, bit
    for bit vs oracle_encode; scale 2^70 pushes coefficients past 2^64 into
    Lattigo's exact big-integer path."""
    torch = torch_cuda
    lib, orc = small
    rng = np.random.default_rng(11)
    level, B = 3, 3
    vals = rng.uniform(-4, 4, (B, orc.N // 2 - 5)).astype(np.float32)
    mods = list(range(level + 1))
    got = lib.export_plaintext(lib.encode_batch(vals, level, 1 << 40))
    for b in range(B):
        assert np.array_equal(got[b], orc.encode(vals[b].astype(np.float64), 2.0 ** 40, mods)), b
    dv = torch.from_numpy(vals).cuda()
    for scale in (2.0 ** 40, 2.0 ** 70):
        got = lib.export_plaintext(lib.encode_batch_device(dv, level, scale))
        for b in range(B):
            assert np.array_equal(got[b], orc.encode(vals[b].astype(np.float64), scale, mods)), (scale, b)


def test_decode_parity(small):
    """GPU decode (INTT, centered CRT, special FFT) vs oracle_decode, bit for
    bit in float64, on decryptions of fresh encryptions."""
    lib, orc = small
    rng = np.random.default_rng(12)
    for level in (0, 4, len(orc.moduli) - orc.K - 1):
        vals = rng.uniform(-2, 2, (2, orc.N // 2)).astype(np.float32)
        dp = lib.Decrypt(lib.Encrypt(lib.encode_batch(vals, level, 1 << 40)))
        got = lib.decode_f64(dp)
        raw = lib.export_plaintext(dp)
        for b in range(2):
            assert np.array_equal(got[b], orc.decode(raw[b], level, 2.0 ** 40)), (level, b)
            assert np.abs(got[b] - vals[b]).max() < 1e-3
        # Decode (Lattigo binding, float32): the same slots rounded to float32
        assert np.array_equal(np.array(lib.Decode(dp), dtype=np.float32), got.reshape(-1).astype(np.float32))


def test_encrypt_parity(small):
    """GPU public-key encryption (ChaCha20 sampler, encoder.hip) vs the oracle's
    restatement with the same seed and encryption index, image by image."""
    lib, orc = small
    rng = np.random.default_rng(13)
    level, B = 4, 2
    vals = rng.uniform(-1, 1, (B, orc.N // 2)).astype(np.float32)
    pt = lib.encode_batch(vals, level, 1 << 40)
    ptv = lib.export_plaintext(pt)
    pk = lib.export_public_key()
    enc = int(lib.OrionHipEncryptionIndex())
    ct = lib.Encrypt(pt)
    assert int(lib.OrionHipEncryptionIndex()) == enc + 1
    got = lib.export_ciphertext(ct)
    for b in range(B):
        assert np.array_equal(got[b], orc.encrypt_pk(1234, enc, b, pk, ptv[b], level)), b


@pytest.mark.parametrize("cheb,coeffs", [
    (True, [0.1, 0.6, 0.0, -0.25, 0.05, 0.3, -0.02, 0.11]),                    # degree 7, depth 3
    (True, list(np.linspace(-0.4, 0.4, 16))),                                   # degree 15, depth 4
    (True, list(0.3 * np.cos(np.arange(32)) / (1 + np.arange(32)))),           # degree 31, depth 5
    (False, [0.5, -1.0, 0.25, 0.125, -0.3, 0.2]),                               # monomial degree 5
    (False, [0.75, 0.5]),                                                       # degree 1
    (True, [0.375]),                                                            # degree 0
])
def test_polynomial_parity(small, cheb, coeffs):
    """EvaluatePolynomial (polyeval.go:63-84) vs the oracle's restatement, bit
    for bit, plus its contract: level - bitlen(degree), exactly the target
    scale, and decrypt ~ p(x)."""
    lib, orc = small
    rng = np.random.default_rng(14)
    level, B = 5, 2
    xs = rng.uniform(-1, 1, (B, orc.N // 2)).astype(np.float32)
    ct = lib.Encrypt(lib.encode_batch(xs, level, 1 << 40))
    x = lib.export_ciphertext(ct)
    cf = np.array(coeffs, dtype=np.float32)
    poly = lib.GenerateChebyshev(list(cf), len(cf)) if cheb else lib.GenerateMonomial(list(cf))
    out = lib.EvaluatePolynomial(ct, poly, 1 << 40)
    depth = int(len(cf) - 1).bit_length()
    assert lib.GetCiphertextLevel(out) == level - depth
    assert lib.GetCiphertextScaleF(out) == 2.0 ** 40
    got = lib.export_ciphertext(out)
    rlk = lib.export_relin_key()
    for b in range(B):
        ref, lv, sc = orc.eval_poly(x[b], level, 2.0 ** 40, cf.astype(np.float64), cheb, 2.0 ** 40, rlk)
        assert lv == level - depth and sc == 2.0 ** 40
        assert np.array_equal(got[b], ref), b
    dec = lib.decode_f64(lib.Decrypt(out))
    xd = xs.astype(np.float64)
    exp = np.polynomial.chebyshev.chebval(xd, cf) if cheb else np.polynomial.polynomial.polyval(xd, cf)
    assert np.abs(dec - exp).max() < 1e-3


def test_polynomial_level_error(small):
    lib, _ = small
    ct = lib.Encrypt(lib.encode_batch(np.zeros((1, 8), np.float32), 1, 1 << 40))
    poly = lib.GenerateMonomial([1.0, 0.5, 0.25, 0.125])  # degree 3: depth 2 > level 1
    with pytest.raises(RuntimeError, match="cannot evaluate poly"):
        lib.EvaluatePolynomial(ct, poly, 1 << 40)


def test_rescale_parity(small):
    lib, orc = small
    rng = np.random.default_rng(3)
    level = 5
    x = rand_ct(rng, orc.moduli, level, orc.N, B=2)
    ct = lib.import_ciphertext(x, 2.0 ** 80)
    lib.Rescale(ct)
    got = lib.export_ciphertext(ct)
    for b in range(2):
        assert np.array_equal(got[b], orc.rescale(x[b], level))
    assert lib.GetCiphertextLevel(ct) == level - 1


def test_mul_relin_parity(small):
    lib, orc = small
    rng = np.random.default_rng(4)
    level = 4
    a = rand_ct(rng, orc.moduli, level, orc.N, B=2)
    b = rand_ct(rng, orc.moduli, level, orc.N, B=2)
    ca, cb = lib.import_ciphertext(a, 2.0 ** 40), lib.import_ciphertext(b, 2.0 ** 40)
    cc = lib.MulRelinCiphertextNew(ca, cb)
    got = lib.export_ciphertext(cc)
    rlk = lib.export_relin_key()
    for i in range(2):
        assert np.array_equal(got[i], orc.mul_relin(a[i], b[i], rlk, level)), i


def test_rotate_parity(small):
    lib, orc = small
    rng = np.random.default_rng(5)
    level = 3
    a = rand_ct(rng, orc.moduli, level, orc.N, B=1)
    ca = lib.import_ciphertext(a, 2.0 ** 40)
    for k in [1, 5, -3, 1000]:
        cr = lib.RotateNew(ca, k)
        g = int(lib.GaloisElement(k))
        assert g == orc.galois_element(k)
        gk = lib.export_galois_key(g)
        got = lib.export_ciphertext(cr)[0]
        assert np.array_equal(got, orc.rotate(a[0], g, gk, level)), k


def test_rotate_decrypts(small):
    lib, orc = small
    rng = np.random.default_rng(6)
    vals = rng.standard_normal(orc.N // 2).astype(np.float32)
    ct = lib.Encrypt(lib.Encode(list(vals), 5, 1 << 40))
    r = lib.RotateNew(ct, 7)
    dec = np.array(lib.Decode(lib.Decrypt(r)))
    assert np.abs(dec - np.roll(vals, -7)).max() < 1e-3


def test_linear_transform_parity(small):
    lib, orc = small
    rng = np.random.default_rng(7)
    slots = orc.N // 2
    level = 4
    idx = [0, 1, 2, 3, 17, 64, 65, 300, slots - 1]
    diags = rng.uniform(-1, 1, (len(idx), slots)).astype(np.float32)
    lt = lib.GenerateLinearTransform(idx, list(diags.reshape(-1)), level, 2.0, "none")
    gels = lib.GetLinearTransformRotationKeys(lt)
    lib.GenerateConsolidatedRotationKeys(gels)
    vals = rng.standard_normal(slots).astype(np.float32)
    ct = lib.Encrypt(lib.Encode(list(vals), level, 1 << 40))
    x = lib.export_ciphertext(ct)[0]
    out = lib.EvaluateLinearTransform(lt, ct)
    got = lib.export_ciphertext(out)[0]
    N1 = lib.GetLinearTransformN1(lt)
    assert N1 == orc.find_best_bsgs_n1(idx, 0)
    pts = [lib.export_lt_diagonal(lt, d, level) for d in idx]
    gkeys = {g: lib.export_galois_key(g) for g in gels if g != 1}
    ref = orc.lt_bsgs(x, level, idx, pts, N1, gkeys)
    assert np.array_equal(got, ref)
    # functional: y[k] = sum_d diag_d[k] * x[k+d]
    lib.Rescale(out)
    dec = np.array(lib.Decode(lib.Decrypt(out)))
    exp = sum(diags[i].astype(np.float64) * np.roll(vals, -d) for i, d in enumerate(idx))
    assert np.abs(dec - exp).max() < 1e-3


def test_lola_n13_end_to_end(torch_cuda):
    """The reference frontend's LoLA op stream (tests/golden/lola_n13_*) replayed
    through the C-ABI: decrypted output vs the cleartext PyTorch model, the
    reference's own numeric gate (tests/models/test_mlp.py:45-48, MAE < 0.005)."""
    from orion_amd.replay import OrionStream
    st = OrionStream("lola_n13", seed=11)
    st.keygen()
    st.compile()
    imgs = np.stack([st.reference_input().reshape(1, 28, 28)] * 3)
    ct = st.encrypt_batch(imgs)
    out = st.forward(ct)
    res = st.decrypt_output(out)
    exp = st.arrays["expected_output"].reshape(-1)
    for b in range(3):
        assert np.abs(res[b] - exp).mean() < 0.005
    # replaying twice gives the same ciphertext (deterministic kernels)
    out2 = st.forward(ct)
    assert np.array_equal(st.lib.export_ciphertext(out), st.lib.export_ciphertext(out2))


def test_lola_n13_matches_cpu_oracle_replay(torch_cuda):
    """Whole-network ciphertext parity: the GPU replay and the CPU-oracle replay
    of the same op stream, same keys and same input ciphertext, bit for bit."""
    from orion_amd.replay import OrionStream
    from oracle.replay_cpu import CpuStream
    st = OrionStream("lola_n13", seed=12)
    st.keygen()
    st.compile()
    lib = st.lib
    cpu = CpuStream("lola_n13")
    # share the GPU's keys with the oracle
    cpu.sk = lib.export_secret_key()
    cpu.rlk = lib.export_relin_key()
    cpu.compile_keys = False
    cpu.gks = {}
    for g in _galois_elements(st):
        cpu.gks[g] = lib.export_galois_key(g)
    cpu.compile()
    ct = st.encrypt_batch(st.reference_input()[None])
    x = lib.export_ciphertext(ct)[0]
    out = lib.export_ciphertext(st.forward(ct))[0]
    enc = [e for e in cpu.trace["events"] if e["phase"] == "input" and e["op"] == "Encode"][0]
    ref = cpu.forward((x, x.shape[1] - 1, float(enc["args"][2])))
    assert np.array_equal(out, ref[0])


def _galois_elements(st):
    lib = st.lib
    gels = set()
    for rid, h in st.lt_map.items():
        gels.update(lib.GetLinearTransformRotationKeys(h))
    for ev in st.trace["events"]:
        if ev["phase"] == "forward" and ev["op"] in ("RotateNew", "Rotate"):
            gels.add(int(lib.GaloisElement(ev["args"][1])))
    return sorted(g for g in gels if g != 1)  # 1: the zero rotation needs no key


def test_n16_ops_parity(torch_cuda, oracle_mod):
    """N = 2^16 (BASELINE config C4's ring degree; its NTT is the two-pass
    kernel): mul_relin, rotate and rescale bit-exact vs the oracle."""
    from orion_amd.backend import HipLibrary
    logq, logp = [60, 40, 40, 40], [60, 60]
    lib = HipLibrary().new_scheme(16, logq, logp, 40, h=192, seed=77)
    mods = lib.moduli()
    orc = oracle_mod.Oracle(16, mods, len(logq), len(logp))
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    rng = np.random.default_rng(16)
    level = 3
    a = rand_ct(rng, mods, level, orc.N, B=2)
    b = rand_ct(rng, mods, level, orc.N, B=2)
    ca, cb = lib.import_ciphertext(a, 2.0 ** 40), lib.import_ciphertext(b, 2.0 ** 40)
    cc = lib.MulRelinCiphertextNew(ca, cb)
    got = lib.export_ciphertext(cc)
    rlk = lib.export_relin_key()
    ref = [orc.mul_relin(a[i], b[i], rlk, level) for i in range(2)]
    for i in range(2):
        assert np.array_equal(got[i], ref[i]), i
    g = int(lib.GaloisElement(3))
    cr = lib.RotateNew(cc, 3)
    gk = lib.export_galois_key(g)
    rot = lib.export_ciphertext(cr)
    for i in range(2):
        assert np.array_equal(rot[i], orc.rotate(ref[i], g, gk, level)), i
    lib.Rescale(cr)
    res = lib.export_ciphertext(cr)
    for i in range(2):
        assert np.array_equal(res[i], orc.rescale(rot[i], level)), i
    # functional: encode -> encrypt -> square -> decrypt at N = 2^16
    vals = rng.standard_normal(orc.N // 2).astype(np.float32)
    pt = lib.Encode(list(vals), level, 1 << 40)
    # the encoder's FFT runs its 3 widest stages in registers at N = 2^16
    assert np.array_equal(lib.export_plaintext(pt)[0],
                          orc.encode(vals.astype(np.float64), 2.0 ** 40, list(range(level + 1))))
    ct = lib.Encrypt(pt)
    sq = lib.MulRelinCiphertextNew(ct, ct)
    lib.Rescale(sq)
    dp = lib.Decrypt(sq)
    dec = lib.decode_f64(dp)[0]
    assert np.array_equal(dec, orc.decode(lib.export_plaintext(dp)[0], level - 1, lib.GetCiphertextScaleF(sq)))
    assert np.abs(dec - vals.astype(np.float64) ** 2).max() < 1e-3
    lib.DeleteScheme()


@pytest.mark.parametrize("cheb,deg,odd", [
    (True, 63, False),   # logSplit 3; the lead node of degree 7 is re-split with logSplit 1
    (True, 27, True),    # odd (a minimax sign stage): even coefficients zero
    (True, 100, False),  # depth 7, non-power-of-two degree
    (False, 40, False),  # monomial basis, depth 6
])
def test_polynomial_parity_deep(torch_cuda, cheb, deg, odd):
    """Deeper Paterson-Stockmeyer trees (recursePS: lead re-split, non-lead
    leaves at several levels, babies up to 2^logSplit - 1) vs the oracle, bit
    for bit, on a 45-bit chain; level - bitlen(degree), the exact target
    scale, decrypt ~ p(x)."""
    from oracle.oracle import Oracle
    from orion_amd.backend import HipLibrary
    logq = [60] + [45] * 9
    lib = HipLibrary().new_scheme(13, logq, [60, 60], 45, h=192, seed=21)
    orc = Oracle(13, lib.moduli(), len(logq), 2)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    rng = np.random.default_rng(deg)
    level, B = 9, 1
    xs = rng.uniform(-1, 1, (B, orc.N // 2)).astype(np.float32)
    ct = lib.Encrypt(lib.encode_batch(xs, level, 1 << 45))
    x = lib.export_ciphertext(ct)
    cf = (rng.uniform(-1, 1, deg + 1) / (1 + np.arange(deg + 1))).astype(np.float32)
    if odd:
        cf[0::2] = 0
    poly = lib.GenerateChebyshev(list(cf), len(cf)) if cheb else lib.GenerateMonomial(list(cf))
    out = lib.EvaluatePolynomial(ct, poly, 1 << 45)
    depth = int(deg).bit_length()
    assert lib.GetCiphertextLevel(out) == level - depth
    assert lib.GetCiphertextScaleF(out) == 2.0 ** 45
    got = lib.export_ciphertext(out)
    ref, lv, sc = orc.eval_poly(x[0], level, 2.0 ** 45, cf.astype(np.float64), cheb, 2.0 ** 45,
                                lib.export_relin_key())
    assert lv == level - depth and sc == 2.0 ** 45
    assert np.array_equal(got[0], ref)
    dec = lib.decode_f64(lib.Decrypt(out))
    xd = xs.astype(np.float64)
    exp = np.polynomial.chebyshev.chebval(xd, cf) if cheb else np.polynomial.polynomial.polyval(xd, cf)
    assert np.abs(dec - exp).max() < 1e-4
    lib.DeleteScheme()


BTP_LOGQ = [60] + [40] * 5  # the residual chain; the bootstrapping chain adds 15 levels above it


@pytest.mark.parametrize("h", [32, 192])
def test_bootstrap_functional(torch_cuda, h):
    """Bootstrap (bootstrapper.go:19-80) of a level-0 batch.  As in Lattigo,
    each slot count gets its own bootstrapper, made once, under bootstrapping
    parameters of its own: the residual Q chain plus the circuit's 15 levels
    (Lattigo's defaults [U]: 4 CoeffsToSlots + 5 polynomial + 3 double-angle
    + 3 SlotsToCoeffs), and P primes of the bit sizes logPs.  The scheme's chain and keys are not
    touched.  The refreshed ciphertext sits on the residual top level at the
    input scale.  A sparse slot count n runs the n-point circuit (trace, one
    packed EvalMod) and Orion's post-scale 2^(LogMaxSlots - LogSlots)
    (bootstrapper.go:73-74): an input whose slots >= n are zero comes back with
    its n slots replicated over all N/2, as Lattigo's sparse packing leaves it.
    Bit parity with Lattigo's own bootstrapper is unpinned (Lattigo is not
    in this image); the bar here is the functional one."""
    from orion_amd.backend import HipLibrary
    lib = HipLibrary().new_scheme(13, BTP_LOGQ, [60, 60], 40, h=h, seed=5)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    n = lib.N // 2
    rng = np.random.default_rng(h)
    vals = rng.uniform(-1, 1, (2, n)).astype(np.float32)
    pre = lib.Encrypt(lib.encode_batch(vals, 3, 1 << 40))
    idx = [0, 3]
    diags = rng.uniform(-1, 1, (2, n)).astype(np.float32)
    lt = lib.GenerateLinearTransform(idx, list(diags.reshape(-1)), 3, 2.0, "none")
    q_before = list(lib.GetModuliChain())
    with pytest.raises(RuntimeError, match="power of two"):
        lib.NewBootstrapper([61, 61], 3 * n // 4)
    lib.NewBootstrapper([61, 61], n)
    lib.NewBootstrapper([55], n)  # bootstrapper.go:25-27: made once per slot count
    assert list(lib.GetModuliChain()) == q_before  # the scheme's parameters are unchanged
    bq, bp = lib.bootstrap_moduli(n)
    assert bq[:len(BTP_LOGQ)] == q_before[:len(BTP_LOGQ)] and len(bq) == len(BTP_LOGQ) + 15
    assert [int(p).bit_length() for p in bp] == [61, 61]  # logPs
    assert len(set(bq + bp + q_before)) == len(bq) + len(bp) + len(q_before) - len(BTP_LOGQ)
    assert all(p % (2 * lib.N) == 1 for p in bq + bp)
    # state from before NewBootstrapper: decrypt, and the transform
    assert np.abs(lib.decode_f64(lib.Decrypt(pre)) - vals).max() < 1e-5
    y = lib.EvaluateLinearTransform(lt, pre)
    lib.Rescale(y)
    exp = sum(diags[i].astype(np.float64) * np.roll(vals, -d, axis=1) for i, d in enumerate(idx))
    assert np.abs(lib.decode_f64(lib.Decrypt(y)) - exp).max() < 1e-3
    ct = lib.Encrypt(lib.encode_batch(vals, 0, 1 << 40))
    out = lib.Bootstrap(ct, n)
    assert lib.GetCiphertextLevel(out) == len(BTP_LOGQ) - 1
    assert lib.GetCiphertextScaleF(out) == 2.0 ** 40
    # the bootstrapping context's launches are in the profile counters (its
    # CoeffsToSlots / SlotsToCoeffs transforms run lt_bsgs; none run outside it here)
    lib.OrionHipProfileReset()
    lib.OrionHipProfile(1)
    lib.DeleteCiphertext(lib.Bootstrap(ct, n))
    lib.OrionHipProfile(0)
    prof = lib.profile_read()
    assert prof["lt_bsgs"]["launches"] > 0 and prof["ntt_fwd"]["ms"] > 0, prof
    dec = lib.decode_f64(lib.Decrypt(out))
    err = np.abs(dec - vals.astype(np.float64))
    # Lattigo's default message ratio (2^8) and degree-30 CosDiscrete cosine:
    # measured 8.5e-8 / 1.3e-8 (h = 32) and 1.0e-7 / 1.3e-8 (h = 192), r05b; the
    # Chebyshev-node cosine of round 4 gave ~1e-5 max
    print("bootstrap full h=%d err max %.3g mean %.3g" % (h, err.max(), err.mean()))
    assert err.max() < 2.5e-7 and err.mean() < 3e-8, (err.max(), err.mean())
    # the refreshed ciphertext computes: square and rescale
    sq = lib.MulRelinCiphertextNew(out, out)
    lib.Rescale(sq)
    d2 = lib.decode_f64(lib.Decrypt(sq))
    assert np.abs(d2 - vals.astype(np.float64) ** 2).max() < 1e-4
    # sparse slot counts (tensors.py:294-305 passes 2^ceil(log2(elements))): slots >= ns
    # zeroed (operations.py:76-84); the output holds the ns slots replicated
    with pytest.raises(RuntimeError, match="no bootstrapper found for slot count"):
        lib.Bootstrap(ct, n // 4)
    for ns, logp in ((n // 4, [61, 61, 61]), (64, [])):
        lib.NewBootstrapper(logp, ns)
        bq2, bp2 = lib.bootstrap_moduli(ns)
        assert [int(p).bit_length() for p in bp2] == (logp or [60, 60])
        sp = vals.copy()
        sp[:, ns:] = 0
        cs = lib.Encrypt(lib.encode_batch(sp, 0, 1 << 40))
        out_s = lib.Bootstrap(cs, ns)
        assert lib.GetCiphertextLevel(out_s) == len(BTP_LOGQ) - 1
        assert lib.GetCiphertextScaleF(out_s) == 2.0 ** 40
        exp_s = np.tile(sp[:, :ns], (1, n // ns)).astype(np.float64)
        err = np.abs(lib.decode_f64(lib.Decrypt(out_s)) - exp_s)
        # the post-scale multiplies the error by the gap (64 at ns = 64); measured
        # (r05b) ns = 1024: 1.3e-7 / 2.2e-8, ns = 64: 6.1e-7 / 1.1e-7 -- bars at ~2x
        print("bootstrap ns=%d h=%d err max %.3g mean %.3g" % (ns, h, err.max(), err.mean()))
        bar = {64: (1.3e-6, 2.2e-7)}.get(ns, (3e-7, 5e-8))
        assert err.max() < bar[0] and err.mean() < bar[1], (ns, err.max(), err.mean())
    lib.DeleteBootstrappers()
    with pytest.raises(RuntimeError, match="no bootstrapper"):
        lib.Bootstrap(ct, n)
    lib.DeleteScheme()


@pytest.mark.parametrize("sparse", [False, True])
def test_bootstrap_parity(torch_cuda, oracle_mod, sparse):
    """Bootstrap bit for bit against the oracle's own
    restatement of Lattigo v6's default bootstrapping circuit
    (oracle_bootstrap: ScaleDown by F, EvkDenseToSparse, centred ModRaise,
    EvkSparseToDense, trace, 4 CoeffsToSlots transforms, conjugation, EvalMod
    = degree-30 CosDiscrete cosine + 3 double angles, 3 SlotsToCoeffs
    transforms, Orion's post-scale).  The oracle derives the prime chain, F,
    K, the cosine coefficients, the trace elements and every CoeffsToSlots /
    SlotsToCoeffs diagonal (special-FFT factorisation, constant spreading,
    packing, BSGS split, encoding at scale q_level over QP) from the
    parameters; only the keys and the input ciphertext are shared.  The two
    derivations are compared item by item first (so a mismatch names its
    constant), then the outputs bit for bit.  Full slots (real and imaginary
    EvalMod) and a sparse slot count (trace, one packed EvalMod); a batch of
    two images."""
    from orion_amd.backend import HipLibrary
    logp = [60, 60]
    lib = HipLibrary().new_scheme(13, BTP_LOGQ, logp, 40, h=192, seed=21)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    n = lib.N // 2
    ns = n // 8 if sparse else n
    lib.NewBootstrapper([61, 61], ns)
    rng = np.random.default_rng(40 + sparse)
    vals = rng.uniform(-1, 1, (2, n)).astype(np.float32)
    vals[:, ns:] = 0
    ct = lib.Encrypt(lib.encode_batch(vals, 0, 1 << 40))
    lib.DeleteCiphertext(lib.Bootstrap(ct, ns))  # every key made at the level it ends at
    out = lib.Bootstrap(ct, ns)
    got, x = lib.export_ciphertext(out), lib.export_ciphertext(ct)
    boot, circ = bootstrap_oracle(oracle_mod, lib, 13, 40, ns, [61, 61])
    # the library's constants against the oracle's own derivation
    lp, op = lib.bootstrap_export(ns, "params"), circ.params()
    for i, name in ((0, "F"), (1, "gap"), (2, "K"), (3, "r"), (4, "degree"), (7, "top")):
        assert int(lp[i]) == int(op[name]), name
    assert lp[6] == op["s_y"] and lp[13] == op["t0"]
    assert np.array_equal(lib.bootstrap_export(ns, "cos"), circ.cos())
    assert sorted(int(g) for g in lib.bootstrap_export(ns, "trace")) == sorted(
        boot.galois_element(ns << i) for i in range(int(op["ntrace"])))
    for k in range(int(op["nlt"])):
        level, n1, idx, diags = circ.lt(k)
        info = lib.bootstrap_export(ns, "lt_info", k)
        assert (int(info[0]), int(info[1]), [int(v) for v in info[3:]]) == (level, n1, idx), k
        for j in range(len(idx)):
            assert np.array_equal(lib.bootstrap_export(ns, "lt_diag", (k << 32) | j).reshape(diags[j].shape),
                                  diags[j]), (k, j)
    keys = bootstrap_keys(lib, ns)
    orc = oracle_mod.Oracle(13, lib.moduli(), len(BTP_LOGQ), len(logp))
    for b in range(2):
        ref, rsc = orc.bootstrap(boot, circ, keys, x[b], 0, 2.0 ** 40)
        assert np.array_equal(got[b], ref), b
    assert lib.GetCiphertextScaleF(out) == 2.0 ** 40 == float(rsc)
    exp = np.tile(vals[:, :ns], (1, n // ns)).astype(np.float64)
    assert np.abs(lib.decode_f64(lib.Decrypt(out)) - exp).max() < 1e-6
    # ScaleDown's F comes from the input's own scale (Lattigo's
    # ScaleDown), so an input at another scale keeps the message ratio; the
    # output scale carries F / F_default
    ct2 = lib.Encrypt(lib.encode_batch(vals, 0, 1 << 38))
    out2 = lib.Bootstrap(ct2, ns)
    x2, got2 = lib.export_ciphertext(ct2), lib.export_ciphertext(out2)
    ref2, rsc2 = orc.bootstrap(boot, circ, keys, x2[0], 0, 2.0 ** 38)
    assert np.array_equal(got2[0], ref2)
    # F is 4x the default's: the output comes back near the default scale (as
    # Lattigo's does), carrying F's rounding
    assert lib.GetCiphertextScaleF(out2) == float(rsc2) and abs(float(rsc2) / 2.0 ** 40 - 1) < 1e-3
    assert np.abs(lib.decode_f64(lib.Decrypt(out2)) - exp).max() < 1e-6
    lib.DeleteScheme()


def test_error_contract(torch_cuda):
    """SURVEY §8b errors: where Lattigo panics (aborting the process), the
    C-ABI returns an error with a last-error string; the library stays usable
    afterwards.  Bad handles, a level-0 rescale, mismatched batches.  Deleting
    a handle twice is a no-op, as in the reference heap (minheap.go:77-81:
    Python frees from __del__ at GC-determined times)."""
    from orion_amd.backend import HipLibrary
    lib = HipLibrary().new_scheme(13, [50, 40, 40], [60], 40, h=64, seed=9, device=0)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    vals = np.linspace(-1, 1, 4096).astype(np.float32)
    ct = lib.Encrypt(lib.Encode(vals, 2, 1 << 40))
    for call in (lambda: lib.RotateNew(9999, 1), lambda: lib.Rescale(9999),
                 lambda: lib.MulRelinCiphertextNew(ct, 9999), lambda: lib.Decrypt(9999)):
        with pytest.raises(RuntimeError):
            call()
    low = lib.Encrypt(lib.Encode(vals, 0, 1 << 40))
    with pytest.raises(RuntimeError, match="level-0"):
        lib.Rescale(low)
    b2 = lib.Encrypt(lib.encode_batch(np.stack([vals, vals]), 2, 1 << 40))
    b3 = lib.Encrypt(lib.encode_batch(np.stack([vals, vals, vals]), 2, 1 << 40))
    with pytest.raises(RuntimeError, match="batch"):
        lib.AddCiphertextNew(b2, b3)
    tmp = lib.RotateNew(ct, 1)
    lib.DeleteCiphertext(tmp)
    lib.DeleteCiphertext(tmp)
    # still usable: the error paths left no device state behind
    out = np.array(lib.Decode(lib.Decrypt(lib.RotateNew(ct, 1))))
    assert np.abs(out[:4096] - np.roll(vals, -1)).max() < 1e-4
    lib.DeleteScheme()


@pytest.mark.parametrize("logn", [13, 15])
def test_prime_sizes_across_f64_boundaries(torch_cuda, oracle_mod, logn):
    """Q primes of 41, 42, 45, 46 and 47 bits: the float64 NTT is
    lazy up to 41-bit moduli and reduces every round above (ntt.hip), and the
    float64 path ends at 46-bit moduli (ORION_F64_BITS, common.h).  NTT/INTT,
    mul_relin, rotate and rescale bit-exact vs the oracle on both sides of
    each boundary."""
    torch = torch_cuda
    from orion_amd.backend import HipLibrary
    logq, logp = [60, 40, 41, 42, 45, 46, 47], [60, 60]
    lib = HipLibrary().new_scheme(logn, logq, logp, 40, h=192, seed=41)
    mods = lib.moduli()
    bits = [q.bit_length() for q in mods]
    # lazy float64 (<= 41 bits), reduced float64 (42..46), the 46-bit edge, integer (>= 47)
    assert min(bits) <= 41 and any(42 <= b <= 46 for b in bits) and 46 in bits and 47 in bits, bits
    orc = oracle_mod.Oracle(logn, mods, len(logq), len(logp))
    N, nl, B = 1 << logn, len(mods), 2
    rng = np.random.default_rng(logn + 100)
    import ctypes
    host = np.stack([rng.integers(0, mods[m], (B, N), dtype=np.uint64) for m in range(nl)])
    host[:, 1, :8] = np.array([mods[m] - 1 for m in range(nl)], dtype=np.uint64)[:, None]  # top residues
    dev = torch.from_numpy(host.view(np.int64).copy()).cuda()
    mods_c = (ctypes.c_int * nl)(*range(nl))
    ptr = ctypes.cast(dev.data_ptr(), ctypes.POINTER(ctypes.c_ulong))
    assert lib.lib.OrionHipNTT(ptr, nl, B, mods_c, 0) == 0
    lib.OrionHipSynchronize()
    fwd = dev.cpu().numpy().view(np.uint64)
    for m in range(nl):
        for b in range(B):
            assert np.array_equal(fwd[m, b], orc.ntt(m, host[m, b])), (bits[m], b)
    assert lib.lib.OrionHipNTT(ptr, nl, B, mods_c, 1) == 0
    lib.OrionHipSynchronize()
    assert np.array_equal(dev.cpu().numpy().view(np.uint64), host)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    level = len(logq) - 1
    a = rand_ct(rng, mods, level, N, B=1)
    b = rand_ct(rng, mods, level, N, B=1)
    cc = lib.MulRelinCiphertextNew(lib.import_ciphertext(a, 2.0 ** 40), lib.import_ciphertext(b, 2.0 ** 40))
    ref = orc.mul_relin(a[0], b[0], lib.export_relin_key(), level)
    assert np.array_equal(lib.export_ciphertext(cc)[0], ref)
    g = int(lib.GaloisElement(7))
    cr = lib.RotateNew(cc, 7)
    ref = orc.rotate(ref, g, lib.export_galois_key(g), level)
    assert np.array_equal(lib.export_ciphertext(cr)[0], ref)
    for lv in range(level, 0, -1):  # every prime is the rescale divisor once
        lib.Rescale(cr)
        ref = orc.rescale(ref, lv)
        assert np.array_equal(lib.export_ciphertext(cr)[0], ref), bits[lv]
    lib.DeleteScheme()


@pytest.mark.parametrize("logn", [15, 16])
def test_ntt_edge_residues(torch_cuda, oracle_mod, logn):
    """Constant limbs 0, 1 and q-1 (and alternating 0 / q-1) through the
    forward and inverse NTT at the bench and ResNet ring degrees, every limb
    of a 60/40-bit chain, vs the oracle."""
    torch = torch_cuda
    from orion_amd.backend import HipLibrary
    import ctypes
    logq = [60, 40, 40]
    lib = HipLibrary().new_scheme(logn, logq, [60, 60], 40)
    mods = lib.moduli()
    orc = oracle_mod.Oracle(logn, mods, len(logq), 2)
    N, nl = 1 << logn, len(mods)
    pats = []
    for m in range(nl):
        q = mods[m]
        alt = np.zeros(N, np.uint64)
        alt[1::2] = q - 1
        pats.append(np.stack([np.zeros(N, np.uint64), np.ones(N, np.uint64), np.full(N, q - 1, np.uint64), alt]))
    host = np.stack(pats)  # [limb][4][N]
    dev = torch.from_numpy(host.view(np.int64).copy()).cuda()
    mods_c = (ctypes.c_int * nl)(*range(nl))
    ptr = ctypes.cast(dev.data_ptr(), ctypes.POINTER(ctypes.c_ulong))
    assert lib.lib.OrionHipNTT(ptr, nl, 4, mods_c, 0) == 0
    lib.OrionHipSynchronize()
    fwd = dev.cpu().numpy().view(np.uint64)
    for m in range(nl):
        for k in range(4):
            assert np.array_equal(fwd[m, k], orc.ntt(m, host[m, k])), (m, k)
    assert not fwd[:, 0].any()  # NTT(0) = 0
    assert lib.lib.OrionHipNTT(ptr, nl, 4, mods_c, 1) == 0
    lib.OrionHipSynchronize()
    assert np.array_equal(dev.cpu().numpy().view(np.uint64), host)
    lib.DeleteScheme()


def test_deep_chain_n16(torch_cuda, oracle_mod):
    """BASELINE config C4's arithmetic at full depth: N = 2^16 with
    configs/resnet.yml's chain ([60] + [30] x 32 Q primes, P = [60, 60], so 17
    gadget digits).  Ten consecutive mul_relin -> rescale steps from the top
    level, then a rotation and a hoisted-BSGS linear transform, each bit-exact
    vs the oracle (two images per launch)."""
    from orion_amd.backend import HipLibrary
    logq, logp = [60] + [30] * 32, [60, 60]
    lib = HipLibrary().new_scheme(16, logq, logp, 30, h=192, seed=161)
    mods = lib.moduli()
    orc = oracle_mod.Oracle(16, mods, len(logq), len(logp))
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    rlk = lib.export_relin_key()
    assert rlk.shape[0] == 17
    rng = np.random.default_rng(1616)
    level, B = len(logq) - 1, 2
    x = rand_ct(rng, mods, level, orc.N, B=B)
    ct = lib.import_ciphertext(x, 2.0 ** 30)
    ref = [x[b] for b in range(B)]
    for step in range(10):
        nxt = lib.MulRelinCiphertextNew(ct, ct)
        lib.Rescale(nxt)
        lib.DeleteCiphertext(ct)
        ct = nxt
        got = lib.export_ciphertext(ct)
        for b in range(B):
            ref[b] = orc.rescale(orc.mul_relin(ref[b], ref[b], rlk, level), level)
            assert np.array_equal(got[b], ref[b]), (step, b)
        level -= 1
    del rlk
    g = int(lib.GaloisElement(5))
    cr = lib.RotateNew(ct, 5)
    gk = lib.export_galois_key(g)
    got = lib.export_ciphertext(cr)
    for b in range(B):
        assert np.array_equal(got[b], orc.rotate(ref[b], g, gk, level)), b
    del gk
    slots = orc.N // 2
    idx = [0, 1, 2, 3, 64, 65, 1000, slots - 1]
    diags = rng.uniform(-1, 1, (len(idx), slots)).astype(np.float32)
    lt = lib.GenerateLinearTransform(idx, list(diags.reshape(-1)), level, 2.0, "none")
    gels = lib.GetLinearTransformRotationKeys(lt)
    lib.GenerateConsolidatedRotationKeys(gels)
    out = lib.export_ciphertext(lib.EvaluateLinearTransform(lt, ct))
    pts = [lib.export_lt_diagonal(lt, d, level) for d in idx]
    gkeys = {e: lib.export_galois_key(e) for e in gels if e != 1}
    N1 = lib.GetLinearTransformN1(lt)
    for b in range(B):
        assert np.array_equal(out[b], orc.lt_bsgs(ref[b], level, idx, pts, N1, gkeys)), b
    lib.DeleteScheme()


def test_basis_extension_modes(torch_cuda, oracle_mod):
    """The four ways a basis-extension target sum is formed (common.h
    BextTarget): ResNet's bootstrapping chain shape ([60] + [30] x 16 Q primes,
    eight 61-bit P primes, so 8-limb gadget digits) puts narrow 30-bit digits
    onto 61-bit P targets (BEXT_WT), the eight P limbs onto 30-bit Q targets in
    every ModDown (BEXT_NT), 30-bit onto 30-bit (BEXT_NARROW), and digit 0
    (with the 60-bit q0) and the q0 target on the lazy path; digits of 8, 3 and
    1 limbs as the level drops.  mul_relin -> rescale steps and rotations,
    bit-exact vs the oracle, with top residues (q - 1) in the inputs."""
    from orion_amd.backend import HipLibrary
    logq, logp = [60] + [30] * 16, [61] * 8
    lib = HipLibrary().new_scheme(13, logq, logp, 30, h=192, seed=77)
    mods = lib.moduli()
    assert [q.bit_length() for q in mods[len(logq):]] == [61] * 8
    orc = oracle_mod.Oracle(13, mods, len(logq), len(logp))
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    rlk = lib.export_relin_key()
    rng = np.random.default_rng(8080)
    level, B = len(logq) - 1, 2
    x = rand_ct(rng, mods, level, orc.N, B=B)
    for m in range(level + 1):
        x[:, :, m, :16] = mods[m] - 1  # top residues in the NTT domain
    ct = lib.import_ciphertext(x, 2.0 ** 30)
    ref = [x[b] for b in range(B)]
    g = int(lib.GaloisElement(3))
    for step in range(8):  # levels 16 -> 8: digits of 8 + 8 + 1, then 8 + 3 limbs
        nxt = lib.MulRelinCiphertextNew(ct, ct)
        lib.Rescale(nxt)
        lib.DeleteCiphertext(ct)
        ct = nxt
        got = lib.export_ciphertext(ct)
        for b in range(B):
            ref[b] = orc.rescale(orc.mul_relin(ref[b], ref[b], rlk, level), level)
            assert np.array_equal(got[b], ref[b]), (step, b)
        level -= 1
        if step in (0, 5):
            cr = lib.RotateNew(ct, 3)
            gk = lib.export_galois_key(g)
            got = lib.export_ciphertext(cr)
            for b in range(B):
                assert np.array_equal(got[b], orc.rotate(ref[b], g, gk, level)), (step, b)
            lib.DeleteCiphertext(cr)
    lib.DeleteScheme()


def test_one_prime_gadget_wide_fused_mac(torch_cuda, oracle_mod, monkeypatch):
    """one P prime (K = 1) makes one gadget digit per Q limb, so a
    16-limb chain has beta = 16; with the INTT fusion unlimited
    (ORION_NTT_IFUSE_MAXR=1000) the key switch takes ks_mac_full_kernel, whose
    LDS is (4 + 2 beta) x 2 KiB = 72 KiB -- past the default 64 KiB a launch
    gets without its attribute.  mul_relin -> rescale at N = 2^15, batch 1
    and 2, bit-exact vs the oracle."""
    monkeypatch.setenv("ORION_NTT_IFUSE_MAXR", "1000")
    from orion_amd.backend import HipLibrary
    logq, logp = [60] + [40] * 15, [61]
    lib = HipLibrary().new_scheme(15, logq, logp, 40, h=192, seed=717)
    mods = lib.moduli()
    orc = oracle_mod.Oracle(15, mods, len(logq), len(logp))
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    rlk = lib.export_relin_key()
    rng = np.random.default_rng(7171)
    level = len(logq) - 1
    for B in (1, 2):
        x = rand_ct(rng, mods, level, orc.N, B=B)
        ct = lib.import_ciphertext(x, 2.0 ** 40)
        cc = lib.MulRelinCiphertextNew(ct, ct)
        lib.Rescale(cc)
        got = lib.export_ciphertext(cc)
        for b in range(B):
            assert np.array_equal(got[b], orc.rescale(orc.mul_relin(x[b], x[b], rlk, level), level)), (B, b)
        lib.DeleteCiphertext(cc)
        lib.DeleteCiphertext(ct)
    lib.DeleteScheme()


@pytest.mark.parametrize("env", [{}, {"ORION_NTT_TAILSPLIT": "1"}, {"ORION_NTT_IFUSE": "0"},
                                 {"ORION_NTT_AUT_FUSE": "0"}, {"ORION_BEXT_MODES": "0", "ORION_NTT_IFUSE_MAXR": "1000"},
                                 {"ORION_NTT_COSPLIT": "0.5", "ORION_NTT_COSPLIT_MIN": "200"},
                                 {"ORION_MODDOWN_LAT": "1"}])
@pytest.mark.parametrize("B", [2, 12, 40])
def test_runtime_switch_parity(torch_cuda, oracle_mod, env, B, monkeypatch):
    """The default environment and the non-default NTT / basis-extension
    paths behind the runtime switches stay bit-exact: the partial-round split (B=40 at
    N=2^15 leaves 144- and 80-job tails), the unfused INTT + prologue NTT,
    the lazy-only basis extension, the INTT fusion with no redundancy limit,
    the rotation's automorphism as its own launch, the one-pass launches
    co-split with the two-pass kernels on CU-masked streams, and every ModDown
    on the fused latency path whatever its size; and the fused
    rotate-and-add (OrionHipRotateAdd) on each of those paths.  B=12 gives
    120-job latency-kernel launches, with more rows-pass workgroups than the
    chip holds at once: a scattering rows pass that stored into rows another
    workgroup has yet to read would show there.  mul_relin -> rescale ->
    rotate on a LoLA-shaped chain; two of the images are checked against the
    oracle."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    from orion_amd.backend import HipLibrary
    logq, logp = [60, 40, 40, 40, 40, 40], [60, 60]
    lib = HipLibrary().new_scheme(15, logq, logp, 40, h=192, seed=515)
    mods = lib.moduli()
    orc = oracle_mod.Oracle(15, mods, len(logq), len(logp))
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    rng = np.random.default_rng(5150 + B)
    level = len(logq) - 1
    x = rand_ct(rng, mods, level, orc.N, B=B)
    ct = lib.import_ciphertext(x, 2.0 ** 40)
    cc = lib.MulRelinCiphertextNew(ct, ct)
    lib.Rescale(cc)
    g = int(lib.GaloisElement(3))
    cr = lib.RotateNew(cc, 3)
    got_m = lib.export_ciphertext(cc)
    got_r = lib.export_ciphertext(cr)
    rlk, gk = lib.export_relin_key(), lib.export_galois_key(g)
    # x += Rotate(x, 3) in one call (the addition in the ModDown's store, or
    # the accumulating automorph launch with ORION_NTT_AUT_FUSE=0)
    lib.OrionHipRotateAdd(cc, 3)
    got_a = lib.export_ciphertext(cc)
    qs = np.array(mods[:level], dtype=np.uint64)[:, None]
    for b in (0, B - 1):
        ref = orc.rescale(orc.mul_relin(x[b], x[b], rlk, level), level)
        assert np.array_equal(got_m[b], ref), b
        rot = orc.rotate(ref, g, gk, level - 1)
        assert np.array_equal(got_r[b], rot), b
        assert np.array_equal(got_a[b], (ref + rot) % qs), b
    lib.DeleteScheme()


@pytest.mark.parametrize("B", [1, 64])
def test_deferred_rotate_add_plain_calls(torch_cuda, oracle_mod, B):
    """The frontend's `out += out.roll(k)` (linear.py:72-73) as the plain
    C-ABI calls it issues -- RotateNew(x, k) -> r, AddCiphertext(x, r),
    DeleteCiphertext(r) -- runs as one key switch with the addition in its
    store (backend.hip Context::Deferred), bit-exact against orc.rotate + add,
    at B=64 (one-pass kernel) and B=1 (latency kernels).  Every way out of
    the deferral computes what the op-by-op calls would: the rotation read
    after the addition, the rotation read before it, the source written
    before the addition, the rotation deleted unread, and RescaleNew's
    copy-on-write result with either handle written afterwards."""
    from orion_amd.backend import HipLibrary
    logq, logp = [60, 40, 40, 40, 40, 40], [60, 60]
    lib = HipLibrary().new_scheme(15, logq, logp, 40, h=192, seed=616)
    mods = lib.moduli()
    orc = oracle_mod.Oracle(15, mods, len(logq), len(logp))
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    rng = np.random.default_rng(6160 + B)
    level = 3
    qs = np.array(mods[:level + 1], dtype=np.uint64)[:, None]
    x = rand_ct(rng, mods, level, orc.N, B=B)
    chk = (0, B - 1)

    def fresh():
        return lib.import_ciphertext(x, 2.0 ** 40)

    k = 512
    g = int(lib.GaloisElement(k))
    lib.AddRotationKey(k)
    gk = lib.export_galois_key(g)
    rot = {b: orc.rotate(x[b], g, gk, level) for b in chk}
    # 1. the frontend's sequence: fused
    a = fresh()
    lib.OrionHipProfileReset()
    lib.OrionHipProfile(1)
    r = lib.RotateNew(a, k)
    assert lib.AddCiphertext(a, r) == a
    lib.DeleteCiphertext(r)
    lib.OrionHipProfile(0)
    prof = lib.profile_read()
    # no separate addition, no separate permutation: both in the ModDown's store
    assert prof["elementwise"]["launches"] == 0 and prof["automorph"]["launches"] == 0, prof
    assert prof["ks_mac"]["launches"] >= 1, prof
    got = lib.export_ciphertext(a)
    for b in chk:
        assert np.array_equal(got[b], (x[b] + rot[b]) % qs), b
    lib.DeleteCiphertext(a)
    # 2. the rotation read after the addition
    a = fresh()
    r = lib.RotateNew(a, k)
    lib.AddCiphertext(a, r)
    gr, ga = lib.export_ciphertext(r), lib.export_ciphertext(a)
    for b in chk:
        assert np.array_equal(gr[b], rot[b]) and np.array_equal(ga[b], (x[b] + rot[b]) % qs), b
    lib.DeleteCiphertext(r)
    lib.DeleteCiphertext(a)
    # 3. the source written before the addition (the rotation sees the old x)
    a = fresh()
    r = lib.RotateNew(a, k)
    lib.MulScalarInt(a, 3)
    lib.AddCiphertext(a, r)
    lib.DeleteCiphertext(r)
    ga = lib.export_ciphertext(a)
    for b in chk:
        assert np.array_equal(ga[b], (x[b] * 3 % qs + rot[b]) % qs), b
    # 4. the rotation deleted unread; metadata reads keep it pending
    r = lib.RotateNew(a, k)
    assert lib.GetCiphertextLevel(r) == level and lib.GetCiphertextBatch(r) == B
    lib.DeleteCiphertext(r)
    assert np.array_equal(lib.export_ciphertext(a), ga)
    # 5. a rotation added into another ciphertext runs on its own
    c = fresh()
    r = lib.RotateNew(a, k)
    lib.AddCiphertext(c, r)
    lib.DeleteCiphertext(r)
    gc = lib.export_ciphertext(c)
    for b in chk:
        assert np.array_equal(gc[b], (x[b] + orc.rotate(ga[b], g, gk, level)) % qs), b
    lib.DeleteCiphertext(a)
    lib.DeleteCiphertext(c)
    # 6. RescaleNew: y shares x's rescaled buffer until one of them is written
    a = fresh()
    y = lib.RescaleNew(a)
    resc = {b: orc.rescale(x[b], level) for b in chk}
    lib.MulScalarInt(a, 5)
    gy, ga = lib.export_ciphertext(y), lib.export_ciphertext(a)
    q1 = qs[:level]
    for b in chk:
        assert np.array_equal(gy[b], resc[b]) and np.array_equal(ga[b], resc[b] * 5 % q1), b
    lib.DeleteCiphertext(y)
    y = lib.RescaleNew(a)
    lib.MulScalarInt(y, 7)
    gy, ga = lib.export_ciphertext(y), lib.export_ciphertext(a)
    q2 = qs[:level - 1]
    for b in chk:
        exp = orc.rescale(resc[b] * 5 % q1, level - 1)
        assert np.array_equal(ga[b], exp) and np.array_equal(gy[b], exp * 7 % q2), b
    lib.DeleteCiphertext(a)
    lib.MulScalarInt(y, 1)  # sole owner now: in place, no copy
    assert np.array_equal(lib.export_ciphertext(y), gy)
    lib.DeleteScheme()
