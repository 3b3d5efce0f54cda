"""GPU tests of the drop-in boundary's contracts: handle heaps,
stream switching, device-resident import/export, the io_mode save/load
paths in Lattigo's wire layout, and the key-bundle header checks."""
import ctypes

import numpy as np
import pytest

from tests.helpers import SMALL, rand_ct, SchemeCache

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
        lib = HipLibrary().new_scheme(SMALL["logn"], SMALL["logq"], SMALL["logp"], 40, h=192, seed=4321)
        orc = oracle_mod.Oracle(SMALL["logn"], lib.moduli(), len(SMALL["logq"]), len(SMALL["logp"]))
        lib.GenerateSecretKey()
        lib.GeneratePublicKey()
        lib.GenerateRelinearizationKey()
        return lib, orc

    return _small_cache.get(make)


def test_handle_heap_lowest_free_reuse(torch_cuda):
    """minheap.go:46-81: Add takes the smallest freed id first, else the next
    new one; Delete of a live id frees it (twice is a no-op); GetLive* lists
    exactly the live ids.  Ciphertext and plaintext heaps are separate."""
    from orion_amd.backend import HipLibrary
    lib = HipLibrary().new_scheme(13, [50, 40, 40], [60], 40, h=64, seed=8)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    pt = lib.encode_batch(np.zeros((1, 8), np.float32), 2, 1 << 40)
    assert pt == 0 and lib.GetLivePlaintexts() == [0]
    ids = [lib.Encrypt(pt) for _ in range(5)]
    assert ids == [0, 1, 2, 3, 4]
    lib.DeleteCiphertext(3)
    lib.DeleteCiphertext(1)
    lib.DeleteCiphertext(1)  # no-op
    assert sorted(lib.GetLiveCiphertexts()) == [0, 2, 4]
    assert lib.Encrypt(pt) == 1  # lowest free first
    assert lib.CloneCiphertext(0) == 3
    assert lib.Negate(2) == 5  # then the next never-used id
    lib.DeleteCiphertext(0)
    assert lib.Encrypt(pt) == 0
    assert sorted(lib.GetLiveCiphertexts()) == [0, 1, 2, 3, 4, 5]
    assert lib.encode_batch(np.zeros((1, 8), np.float32), 2, 1 << 40) == 1
    lib.DeletePlaintext(0)
    assert lib.GetLivePlaintexts() == [1]
    lib.DeleteScheme()


def test_pool_stats_reuse(torch_cuda):
    """OrionHipPoolStats: the device pools cache freed buffers by size, so a
    second identical op reuses them (no new hipMalloc); held >= cached and the
    peak bounds the held bytes; no forced trim happens at this size."""
    from orion_amd.backend import HipLibrary
    lib = HipLibrary().new_scheme(13, [50, 40, 40], [60], 40, h=64, seed=9)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    ct = lib.Encrypt(lib.encode_batch(np.ones((2, 8), np.float32), 2, 1 << 40))
    lib.DeleteCiphertext(lib.MulRelinCiphertextNew(ct, ct))  # warm the size classes
    a = lib.pool_stats()
    lib.DeleteCiphertext(lib.MulRelinCiphertextNew(ct, ct))
    b = lib.pool_stats()
    assert b["hipmalloc_calls"] == a["hipmalloc_calls"], (a, b)
    assert b["trims"] == a["trims"] and 0 < b["cached_bytes"] <= b["held_bytes"] <= b["peak_bytes"], b
    lib.DeleteScheme()


def test_stream_switch_bit_exact(small, torch_cuda):
    """OrionHipSetStream between two ops (the pool reuses buffers
    across streams): the old stream is drained at the switch, so a result
    computed across switches equals the one computed on one stream."""
    torch = torch_cuda
    lib, orc = small
    rng = np.random.default_rng(21)
    level = 4
    a = rand_ct(rng, orc.moduli, level, orc.N, B=3)
    ca = lib.import_ciphertext(a, 2.0 ** 40)
    ref = lib.export_ciphertext(lib.RotateNew(lib.MulRelinCiphertextNew(ca, ca), 5))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    try:
        for _ in range(3):
            lib.OrionHipSetStream(s1.cuda_stream)
            sq = lib.MulRelinCiphertextNew(ca, ca)
            lib.OrionHipSetStream(s2.cuda_stream)
            r = lib.RotateNew(sq, 5)
            lib.DeleteCiphertext(sq)  # its buffer returns to the pool while s2 may still run
            lib.OrionHipSetStream(None)
            junk = lib.MulRelinCiphertextNew(ca, ca)  # reuses the freed buffer on a new stream
            assert np.array_equal(lib.export_ciphertext(r), ref)
            lib.DeleteCiphertext(junk)
            lib.DeleteCiphertext(r)
    finally:
        lib.OrionHipSetStream(None)


def test_device_import_export(small, torch_cuda):
    """SURVEY §8b device data: ciphertexts imported from / exported to torch
    device tensors ([B][2][level+1][N]) without a host round trip, equal to
    the host path bit for bit, including a rescaled ciphertext whose limb
    planes were allocated for a higher level."""
    torch = torch_cuda
    lib, orc = small
    rng = np.random.default_rng(22)
    level, B = 3, 2
    x = rand_ct(rng, orc.moduli, level, orc.N, B=B)
    d = torch.from_numpy(x.view(np.int64).copy()).cuda()
    h = lib.import_ciphertext_device(d, 2.0 ** 80)
    assert lib.GetCiphertextLevel(h) == level and lib.GetCiphertextBatch(h) == B
    assert np.array_equal(lib.export_ciphertext(h), x)
    lib.Rescale(h)
    ref = lib.export_ciphertext(h)
    out = torch.empty((B, 2, level, orc.N), dtype=torch.int64, device="cuda")
    lib.export_ciphertext_device(h, out)
    lib.OrionHipSynchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint64), ref)
    # no manual synchronisation -- the wrappers order the library
    # stream after the torch work that produces the input (a kernel on the
    # current stream, freed right away: record_stream keeps its memory from
    # being reused before the copy), and torch's readers after the export
    for _ in range(3):
        d2 = d.clone()
        h2 = lib.import_ciphertext_device(d2, 2.0 ** 80)
        del d2
        junk = torch.full_like(d, -1)  # would take d2's memory if the allocator recycled it early
        out2 = torch.zeros_like(d)
        lib.export_ciphertext_device(h2, out2)
        assert np.array_equal((out2 + 0).cpu().numpy().view(np.uint64), x)
        del junk
        lib.DeleteCiphertext(h2)
    with pytest.raises(RuntimeError, match="size mismatch"):
        lib.export_ciphertext_device(h, torch.empty((B, 2, level + 1, orc.N), dtype=torch.int64, device="cuda"))


def test_import_level_checks(small):
    """an import at level >= L (or B < 1) is refused instead of
    handing later ops limbs past the Q chain."""
    lib, orc = small
    L = len(orc.moduli) - orc.K
    bad = np.zeros((1, 2, L + 1, orc.N), np.uint64)
    with pytest.raises(RuntimeError, match="invalid level"):
        lib.import_ciphertext(bad, 1.0)
    with pytest.raises(RuntimeError, match="invalid level"):
        lib.import_plaintext(np.zeros((1, L + 1, orc.N), np.uint64), 1.0)


def _mform(x, q):
    return (int(x) << 64) % q


def test_wire_format_secret_key(small):
    """keygenerator.go:38-58: rlwe.SecretKey MarshalBinary layout (ringqp.Poly:
    ring.Poly Q then P, each a Matrix[uint64] of RNS rows), coefficients in
    Montgomery form; LoadSecretKey(SerializeSecretKey()) is the identity."""
    lib, orc = small
    sk = lib.export_secret_key()
    blob, _ = lib.SerializeSecretKey()
    N, L, K = orc.N, len(orc.moduli) - orc.K, orc.K
    assert len(blob) == (8 + L * (8 + 8 * N)) + (8 + K * (8 + 8 * N))
    w = blob.view(np.uint64)
    assert w[0] == L and w[1] == N
    mods = orc.moduli
    for j in (0, 7, N - 1):
        assert int(w[2 + j]) == _mform(sk[0, j], mods[0])
    p_off = (8 + L * (8 + 8 * N)) // 8
    assert w[p_off] == K and w[p_off + 1] == N
    assert int(w[p_off + 2 + 5]) == _mform(sk[L, 5], mods[L])
    lib.LoadSecretKey(blob)
    assert np.array_equal(lib.export_secret_key(), sk)
    with pytest.raises(RuntimeError, match="truncated|RNS limbs"):
        lib.LoadSecretKey(blob[:-8])


def test_wire_format_rotation_key_and_diagonals(small):
    """lineartransform.go:131-200: GenerateAndSerializeRotationKey marshals a
    fresh rlwe.GaloisKey without keeping it; LoadRotationKey brings it back;
    SerializeDiagonal marshals the ringqp.Poly and drops the diagonal from the
    transform; LoadPlaintextDiagonal restores it and the transform gives the
    same ciphertext."""
    lib, orc = small
    N, L, K = orc.N, len(orc.moduli) - orc.K, orc.K
    dnum = (L + K - 1) // K
    g = int(lib.GaloisElement(9))
    blob, _ = lib.GenerateAndSerializeRotationKey(g)
    with pytest.raises(RuntimeError, match="no galois key"):
        lib.export_galois_key(g)
    w = blob.view(np.uint64)
    assert list(w[:4]) == [g, 2 * N, 0, dnum]
    qp = (8 + L * (8 + 8 * N)) + (8 + K * (8 + 8 * N))
    assert len(blob) == 32 + dnum * (16 + 2 * qp)
    lib.LoadRotationKey(blob, g)
    gk = lib.export_galois_key(g)
    assert w[6] == L and w[7] == N and int(w[8 + 3]) == _mform(gk[0, 0, 0, 3], orc.moduli[0])
    blob2, _ = lib.GenerateAndSerializeRotationKey(g)  # a kept key is left in place
    assert np.array_equal(lib.export_galois_key(g), gk)
    with pytest.raises(RuntimeError, match="Galois element"):
        lib.LoadRotationKey(blob2, int(lib.GaloisElement(3)))

    rng = np.random.default_rng(23)
    slots, level = N // 2, 3
    idx = [0, 5, 40, slots - 2]
    diags = rng.uniform(-1, 1, (len(idx), slots)).astype(np.float32)
    lt = lib.GenerateLinearTransform(idx, list(diags.reshape(-1)), level, 2.0, "save")
    lib.GenerateConsolidatedRotationKeys(lib.GetLinearTransformRotationKeys(lt))
    ct = lib.Encrypt(lib.Encode(list(rng.standard_normal(slots).astype(np.float32)), level, 1 << 40))
    ref = lib.export_ciphertext(lib.EvaluateLinearTransform(lt, ct))
    pts = {d: lib.export_lt_diagonal(lt, d, level) for d in idx}
    blobs = {d: lib.SerializeDiagonal(lt, d)[0] for d in idx}
    for d in idx:
        assert len(blobs[d]) == (8 + (level + 1) * (8 + 8 * N)) + (8 + K * (8 + 8 * N))
    with pytest.raises(RuntimeError, match="not loaded"):
        lib.EvaluateLinearTransform(lt, ct)
    for d in idx:
        lib.LoadPlaintextDiagonal(blobs[d], lt, d)
        assert np.array_equal(lib.export_lt_diagonal(lt, d, level), pts[d])
    assert np.array_equal(lib.export_ciphertext(lib.EvaluateLinearTransform(lt, ct)), ref)

    # io_mode "load" (lineartransform.go:79-88): no diagonal is encoded at
    # generation; the BSGS index and N1 still come from the index list
    lt2 = lib.GenerateLinearTransform(idx, [], level, 2.0, "load")
    assert lib.GetLinearTransformN1(lt2) == lib.GetLinearTransformN1(lt)
    assert sorted(lib.GetLinearTransformRotationKeys(lt2)) == sorted(lib.GetLinearTransformRotationKeys(lt))
    with pytest.raises(RuntimeError, match="not loaded"):
        lib.EvaluateLinearTransform(lt2, ct)
    for d in idx:
        lib.LoadPlaintextDiagonal(blobs[d], lt2, d)
    assert np.array_equal(lib.export_ciphertext(lib.EvaluateLinearTransform(lt2, ct)), ref)

    # a transform's key is serialised full-chain, as Lattigo's
    # GenGaloisKeyNew marshals it, and scoped to the transform's level at load
    gels = [ge for ge in lib.GetLinearTransformRotationKeys(lt) if ge != 1]
    for ge in gels:
        kb, _ = lib.GenerateAndSerializeRotationKey(ge)
        kw = kb.view(np.uint64)
        assert list(kw[:4]) == [ge, 2 * N, 0, dnum] and kw[6] == L
        lib.LoadRotationKey(kb, ge)
        assert lib.GetGaloisKeyLevel(ge) == level
    x = lib.export_ciphertext(ct)[0]
    got = lib.export_ciphertext(lib.EvaluateLinearTransform(lt, ct))[0]
    gkeys = {ge: lib.export_galois_key(ge) for ge in gels}
    assert np.array_equal(got, orc.lt_bsgs(x, level, idx, [pts[d] for d in idx], lib.GetLinearTransformN1(lt), gkeys))

    # a key cut at load to its transform's level comes back whole -- the
    # loaded key itself, which stays in host memory as Lattigo keeps it
    # (lineartransform.go:143-159) -- for a rotation above that level
    ge = gels[-1]
    k = next(r for r in range(slots) if pow(5, r, 2 * N) == ge)
    kb, _ = lib.GenerateAndSerializeRotationKey(ge)
    lib.LoadRotationKey(kb, ge)
    assert lib.GetGaloisKeyLevel(ge) == level
    top = L - 1
    y = rand_ct(rng, orc.moduli, top, N, B=1)
    r = lib.export_ciphertext(lib.RotateNew(lib.import_ciphertext(y, 2.0 ** 40), k))[0]
    assert lib.GetGaloisKeyLevel(ge) == top
    gk = lib.export_galois_key(ge)
    kw = kb.view(np.uint64)
    for d in range(dnum):
        for c in range(2):
            # digit d, component c: its Q poly's top limb in the blob (Montgomery form)
            off = 4 + 2 + d * (2 + 2 * (2 + (L + K) * (1 + N))) + c * (2 + (L + K) * (1 + N)) + 1 + top * (1 + N) + 1
            for n in (0, 1, N // 3, N - 1):
                assert int(kw[off + n]) == _mform(gk[d, c, top, n], orc.moduli[top]), (d, c, n)
    assert np.array_equal(r, orc.rotate(y[0], ge, gk, top))


def test_key_bundle_header_checks(torch_cuda):
    """the key bundle names its chain (logN, L, K, dnum, moduli);
    a bundle from another chain and a truncated bundle are refused."""
    torch = torch_cuda
    from orion_amd.backend import HipLibrary
    lib = HipLibrary().new_scheme(13, [50, 40, 40], [60], 40, h=64, seed=3)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    lib.AddRotationKey(1)
    n = lib.KeyBundleBytes(0)
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    assert lib.lib.ExportKeyBundle(buf.data_ptr(), 0) == 0
    assert lib.lib.ImportKeyBundle(buf.data_ptr(), 16) != 0
    assert "shorter" in lib.lib.OrionHipLastError().decode()
    assert lib.lib.ImportKeyBundle(buf.data_ptr(), n - 8) != 0
    assert "truncated" in lib.lib.OrionHipLastError().decode()
    assert lib.lib.ImportKeyBundle(buf.data_ptr(), n) == 0
    lib.DeleteScheme()
    lib.new_scheme(13, [50, 40, 40, 40], [60], 40, h=64, seed=3)
    assert lib.lib.ImportKeyBundle(buf.data_ptr(), n) != 0
    assert "another modulus chain" in lib.lib.OrionHipLastError().decode()
    lib.DeleteScheme()


def test_level_scoped_galois_keys(torch_cuda, oracle_mod):
    """A rotation key asked for by a linear transform is made for that
    transform's level (ceil((l+1)/K) digits over l+1+K limbs), so keys of
    low-level transforms stay small under a long chain; a later use at a
    higher level replaces it with a key for that level.  Results stay
    bit-exact vs the oracle either way, and the key bundle carries each
    key's level."""
    torch = torch_cuda
    from orion_amd.backend import HipLibrary
    logq, logp = [55] + [40] * 7, [60, 60]
    lib = HipLibrary().new_scheme(13, logq, logp, 40, h=192, seed=77)
    mods = lib.moduli()
    orc = oracle_mod.Oracle(13, mods, len(logq), len(logp))
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    slots, lt_level = orc.N // 2, 2
    rng = np.random.default_rng(30)
    idx = [0, 3, 9, 40]
    diags = rng.uniform(-1, 1, (len(idx), slots)).astype(np.float32)
    lt = lib.GenerateLinearTransform(idx, list(diags.reshape(-1)), lt_level, 2.0, "none")
    gels = lib.GetLinearTransformRotationKeys(lt)
    lib.GenerateConsolidatedRotationKeys(gels)
    for g in gels:
        if g != 1:  # the zero rotation has no key
            assert lib.GetGaloisKeyLevel(g) == lt_level
    x = rand_ct(rng, mods, lt_level, orc.N, B=1)
    out = lib.export_ciphertext(lib.EvaluateLinearTransform(lt, lib.import_ciphertext(x, 2.0 ** 40)))[0]
    pts = [lib.export_lt_diagonal(lt, d, lt_level) for d in idx]
    gkeys = {g: lib.export_galois_key(g) for g in gels if g != 1}
    N1 = lib.GetLinearTransformN1(lt)
    assert np.array_equal(out, orc.lt_bsgs(x[0], lt_level, idx, pts, N1, gkeys))
    # a rotation by one of the transform's steps, at the top level: the key is remade for it
    k = next(r for r in (3, 9, 40, 8, 1, 2) if int(lib.GaloisElement(r)) in gkeys)
    g = int(lib.GaloisElement(k))
    top = len(logq) - 1
    y = rand_ct(rng, mods, top, orc.N, B=1)
    r = lib.export_ciphertext(lib.RotateNew(lib.import_ciphertext(y, 2.0 ** 40), k))[0]
    assert lib.GetGaloisKeyLevel(g) == top
    assert np.array_equal(r, orc.rotate(y[0], g, lib.export_galois_key(g), top))
    # the bundle keeps every key at its level
    levels = {e: lib.GetGaloisKeyLevel(e) for e in gkeys}
    keys = {e: lib.export_galois_key(e) for e in gkeys}
    n = lib.KeyBundleBytes(0)
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    assert lib.lib.ExportKeyBundle(buf.data_ptr(), 0) == 0
    lib.DeleteScheme()
    lib.new_scheme(13, logq, logp, 40, h=192, seed=78)
    assert lib.lib.ImportKeyBundle(buf.data_ptr(), n) == 0, lib.lib.OrionHipLastError()
    for e in gkeys:
        assert lib.GetGaloisKeyLevel(e) == levels[e]
        assert np.array_equal(lib.export_galois_key(e), keys[e])
    lib.DeleteScheme()


def test_graph_capture_replay(torch_cuda):
    """OrionHipGraphBegin/End/Launch: the LoLA N=2^13 forward pass captured
    into one hipGraph replays bit for bit like the stream-launched pass, again
    and again; ciphertexts made after the capture (the pool pins the graph's
    buffers) are not touched by a replay; a capture that would synchronise
    (an upload) fails with an error instead of recording a broken graph."""
    from orion_amd.replay import OrionStream
    st = OrionStream("lola_n13", seed=77)
    st.keygen()
    st.compile()
    lib = st.lib
    rng = np.random.default_rng(5)
    imgs = rng.standard_normal((3,) + st.reference_input().shape[1:]).astype(np.float32)
    imgs[0] = st.reference_input()[0]
    ct = st.encrypt_batch(imgs)
    ref_h = st.forward(ct)
    ref = lib.export_ciphertext(ref_h)
    gid, out = st.capture(ct)
    assert gid >= 0
    x = lib.export_ciphertext(ct)
    bystander = lib.import_ciphertext(x, 2.0 ** 26)  # allocated after the capture
    for _ in range(3):
        lib.OrionHipGraphLaunch(gid)
        lib.OrionHipSynchronize()
        assert np.array_equal(lib.export_ciphertext(out), ref)
        assert np.array_equal(lib.export_ciphertext(bystander), x)
        assert np.array_equal(lib.export_ciphertext(ct), x)  # the input is not consumed
    res = st.decrypt_output(out)
    assert np.abs(res[0] - st.arrays["expected_output"].reshape(-1)).mean() < 0.005
    lib.OrionHipGraphDestroy(gid)
    # calls that synchronise are refused inside a capture, before they reach
    # HIP, so the capture stays valid and the library stays usable
    ref_r = lib.export_ciphertext(lib.RotateNew(ct, 5))  # makes the key before the capture
    lib.OrionHipGraphBegin()
    with pytest.raises(RuntimeError, match="not allowed while capturing"):
        lib.import_ciphertext(x, 2.0 ** 26)
    with pytest.raises(RuntimeError, match="not allowed while capturing"):
        lib.Decrypt(ct)
    r = lib.RotateNew(ct, 5)  # recorded, not run
    g2 = lib.OrionHipGraphEnd()
    lib.OrionHipGraphLaunch(g2)
    lib.OrionHipSynchronize()
    assert np.array_equal(lib.export_ciphertext(r), ref_r)
    lib.OrionHipGraphDestroy(g2)
    again = st.forward(ct)
    assert np.array_equal(lib.export_ciphertext(again), ref)
    # buffers a graph reads stay its own: a handle made before the capture and
    # deleted inside it, or deleted after it, does not hand its buffer to a
    # later allocation while the graph can replay
    ref_add = lib.export_ciphertext(lib.AddCiphertextNew(ct, ct))
    y = lib.export_ciphertext(lib.MulScalarIntNew(ct, 3))
    pre, pre2 = lib.CloneCiphertext(ct), lib.CloneCiphertext(ct)
    lib.OrionHipGraphBegin()
    r3 = lib.AddCiphertextNew(pre, pre)
    lib.DeleteCiphertext(pre)  # predates the capture, released inside it
    r4 = lib.AddCiphertextNew(pre2, pre2)
    # in-place ops on handles older than the capture would be reapplied by every replay
    with pytest.raises(RuntimeError, match="predates the graph capture"):
        lib.Rescale(ct)
    with pytest.raises(RuntimeError, match="predates the graph capture"):
        lib.AddCiphertext(pre2, ct)
    g3 = lib.OrionHipGraphEnd()
    lib.DeleteCiphertext(pre2)  # deleted after the capture
    bys = [lib.import_ciphertext(y, 2.0 ** 26) for _ in range(3)]
    for _ in range(2):
        lib.OrionHipGraphLaunch(g3)
        lib.OrionHipSynchronize()
        assert np.array_equal(lib.export_ciphertext(r3), ref_add)
        assert np.array_equal(lib.export_ciphertext(r4), ref_add)
        for b in bys:
            assert np.array_equal(lib.export_ciphertext(b), y)
    lib.OrionHipGraphDestroy(g3)
    lib.DeleteScheme()
