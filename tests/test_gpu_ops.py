"""GPU parity tests of the coefficient-wise evaluator ops and of whole op
streams at the BASELINE configs.

* ct+ct, ct-ct, -ct, ct+pt, ct-pt, ct*pt, ct+scalar, ct*int, ct*float and
  CloneCiphertext (/root/reference/orion/backend/lattigo/evaluator.go:48-294,
  tensors.go / tensors.py:229), checked bit for bit against a numpy
  restatement of the same modular arithmetic (integers, exact);
* MLP N=2^14 (BASELINE config C2) and LoLA N=2^15 (C3): the reference
  frontend's op stream replayed on the GPU and on the CPU oracle with the same
  keys and input ciphertext, compared bit for bit;
* size-independent properties at the full C3 size: batch invariance (every
  image of a batch equals the single-image run) and the key bundle that
  bench.py broadcasts over RCCL (export -> fresh scheme -> import).
"""
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
        lib = HipLibrary().new_scheme(SMALL["logn"], SMALL["logq"], SMALL["logp"], 40, h=192, seed=4321)
        mods = lib.moduli()
        orc = oracle_mod.Oracle(SMALL["logn"], mods, len(SMALL["logq"]), len(SMALL["logp"]))
        return lib, orc

    return _small_cache.get(make)


def _q(orc, level):
    return np.array(orc.moduli[:level + 1], dtype=np.uint64)[:, None]


def _add(a, b, q):
    s = a + b
    return np.where(s >= q, s - q, s)


def _sub(a, b, q):
    return np.where(a >= b, a - b, a + q - b)


def _mul_int(a, k, orc, level):
    """a * k mod q_j per limb (exact, Python ints)."""
    out = np.empty_like(a)
    for j in range(level + 1):
        qj = orc.moduli[j]
        kj = k % qj
        out[..., j, :] = np.array([(int(x) * kj) % qj for x in a[..., j, :].reshape(-1)],
                                  dtype=np.uint64).reshape(a[..., j, :].shape)
    return out


def _round_half_away(x):
    """round-half-away-from-zero of an exact rational (backend.hip add_scalar / mul_float)."""
    from fractions import Fraction
    x = Fraction(x)
    return -int(-x + Fraction(1, 2)) if x < 0 else int(x + Fraction(1, 2))


def test_ct_ct_ops(small):
    lib, orc = small
    rng = np.random.default_rng(21)
    level = 4
    q = _q(orc, level)
    a = rand_ct(rng, orc.moduli, level, orc.N, B=2)
    b = rand_ct(rng, orc.moduli, level, orc.N, B=2)
    ca, cb = lib.import_ciphertext(a, 2.0 ** 40), lib.import_ciphertext(b, 2.0 ** 40)
    assert np.array_equal(lib.export_ciphertext(lib.AddCiphertextNew(ca, cb)), _add(a, b, q))
    assert np.array_equal(lib.export_ciphertext(lib.SubCiphertextNew(ca, cb)), _sub(a, b, q))
    cl = lib.CloneCiphertext(ca)
    assert np.array_equal(lib.export_ciphertext(cl), a)
    neg = lib.Negate(cl)  # a new ciphertext: Evaluator.MulNew(ct, -1.0) (evaluator.go:48-58)
    assert neg != cl
    assert np.array_equal(lib.export_ciphertext(neg), _sub(np.zeros_like(a), a, q))
    # in place, returns its input id (evaluator.go:251-257)
    assert lib.AddCiphertext(ca, cb) == ca
    assert np.array_equal(lib.export_ciphertext(ca), _add(a, b, q))


def test_ct_pt_ops(small):
    lib, orc = small
    rng = np.random.default_rng(22)
    level = 3
    q = _q(orc, level)
    a = rand_ct(rng, orc.moduli, level, orc.N, B=2)
    p = np.stack([rng.integers(0, orc.moduli[j], orc.N, dtype=np.uint64) for j in range(level + 1)])
    ca = lib.import_ciphertext(a, 2.0 ** 40)
    cp = lib.import_plaintext(p, 2.0 ** 40)
    add = lib.export_ciphertext(lib.AddPlaintextNew(ca, cp))
    assert np.array_equal(add[:, 0], _add(a[:, 0], p[None], q)) and np.array_equal(add[:, 1], a[:, 1])
    sub = lib.export_ciphertext(lib.SubPlaintextNew(ca, cp))
    assert np.array_equal(sub[:, 0], _sub(a[:, 0], p[None], q)) and np.array_equal(sub[:, 1], a[:, 1])
    mul = lib.MulPlaintextNew(ca, cp)
    got = lib.export_ciphertext(mul)
    mods = list(range(level + 1))
    for bi in range(2):
        for c in range(2):
            assert np.array_equal(got[bi, c], orc.mul_coeffs(a[bi, c], p, mods)), (bi, c)
    assert lib.GetCiphertextScaleF(mul) == 2.0 ** 80


def test_mod_drop_and_poly_depth(small):
    """evaluator.py:30-41 mod_drop through the HEonGPU-style private call, and
    poly_evaluator.py:58-59 GetPolyDepth."""
    lib, orc = small
    rng = np.random.default_rng(25)
    a = rand_ct(rng, orc.moduli, 4, orc.N, B=1)
    ca = lib.import_ciphertext(a, 2.0 ** 40)
    assert lib._ModDropCiphertext(lib.arithmeticoperator_handle, ca, None) == ca
    assert lib.GetCiphertextLevel(ca) == 3 and lib.GetCiphertextScaleF(ca) == 2.0 ** 40
    assert np.array_equal(lib.export_ciphertext(ca)[0], a[0][:, :4])
    for deg, depth in [(0, 0), (1, 1), (7, 3), (8, 4), (31, 5)]:
        assert lib.GetPolyDepth(lib.GenerateMonomial([0.5] * (deg + 1))) == depth


def test_scale_matching_add(small):
    """Lower-scale operand multiplied by the integer scale ratio before the add."""
    lib, orc = small
    rng = np.random.default_rng(23)
    level = 3
    q = _q(orc, level)
    a = rand_ct(rng, orc.moduli, level, orc.N, B=1)
    p = np.stack([rng.integers(0, orc.moduli[j], orc.N, dtype=np.uint64) for j in range(level + 1)])
    ca = lib.import_ciphertext(a, 2.0 ** 60)
    cp = lib.import_plaintext(p, 2.0 ** 40)
    got = lib.export_ciphertext(lib.AddPlaintextNew(ca, cp))
    pr = _mul_int(p, 1 << 20, orc, level)
    assert np.array_equal(got[0, 0], _add(a[0, 0], pr, q)) and np.array_equal(got[0, 1], a[0, 1])


def test_scalar_ops(small):
    lib, orc = small
    rng = np.random.default_rng(24)
    level = 4
    q = _q(orc, level)
    a = rand_ct(rng, orc.moduli, level, orc.N, B=2)
    scale = 2.0 ** 40
    ca = lib.import_ciphertext(a, scale)
    # AddScalar: round(v * scale) added to every NTT slot of c0 (evaluator.go:102-119)
    v = np.float32(-0.8125)
    from fractions import Fraction
    k = _round_half_away(Fraction(float(v)) * Fraction(scale))
    got = lib.export_ciphertext(lib.AddScalarNew(ca, float(v)))
    kv = np.array([k % m for m in orc.moduli[:level + 1]], dtype=np.uint64)[:, None]
    assert np.array_equal(got[:, 0], _add(a[:, 0], kv[None], q)) and np.array_equal(got[:, 1], a[:, 1])
    # MulScalarInt (evaluator.go:142-159)
    got = lib.export_ciphertext(lib.MulScalarIntNew(ca, -7))
    assert np.array_equal(got, _mul_int(a, -7, orc, level))
    # MulScalarFloat: non-integer constant scaled by q_level, scale grows by q_level
    fv = np.float32(0.37)
    ql = orc.moduli[level]
    kf = _round_half_away(Fraction(float(fv)) * ql)
    m = lib.MulScalarFloatNew(ca, float(fv))
    assert np.array_equal(lib.export_ciphertext(m), _mul_int(a, kf, orc, level))
    assert abs(lib.GetCiphertextScaleF(m) / (scale * ql) - 1) < 1e-12


def _replay_gpu_vs_cpu(name, seed):
    from oracle.replay_cpu import CpuStream
    from orion_amd.replay import OrionStream
    st = OrionStream(name, seed=seed)
    st.keygen()
    st.compile()
    lib = st.lib
    cpu = CpuStream(name)
    cpu.sk = lib.export_secret_key()
    cpu.rlk = lib.export_relin_key()
    gels = set()
    for h in st.lt_map.values():
        gels.update(lib.GetLinearTransformRotationKeys(h))
    for ev in st.trace["events"]:
        if ev["phase"] == "forward" and ev["op"] in ("RotateNew", "Rotate"):
            gels.add(int(lib.GaloisElement(ev["args"][1])))
    cpu.gks = {g: lib.export_galois_key(g) for g in sorted(gels) if g != 1}  # 1: zero rotation, no key
    cpu.compile()
    ct = st.encrypt_batch(st.reference_input()[None])
    x = lib.export_ciphertext(ct)[0]
    out = st.forward(ct)
    got = lib.export_ciphertext(out)[0]
    enc = [e for e in cpu.trace["events"] if e["phase"] == "input" and e["op"] == "Encode"][0]
    ref = cpu.forward((x, x.shape[1] - 1, float(enc["args"][2])))
    assert np.array_equal(got, ref[0])
    res = st.decrypt_output(out)
    exp = st.arrays["expected_output"].reshape(-1)
    assert np.abs(res[0] - exp).mean() < 0.005  # tests/models/test_mlp.py:45-48
    lib.DeleteScheme()


def test_mlp_n13_c1_matches_cpu_oracle_replay(torch_cuda):
    """BASELINE config C1 (configs/mlp.yml, N=2^13, 6 Q + 2 P primes of 26-29
    bits): whole forward pass on the GPU bit for bit vs the oracle, MAE gate."""
    _replay_gpu_vs_cpu("mlp_n13", seed=36)


def test_mlp_n14_matches_cpu_oracle_replay(torch_cuda):
    """BASELINE config C2 (MLP, N=2^14, 8 Q + 2 P primes): whole forward pass."""
    _replay_gpu_vs_cpu("mlp_n14", seed=31)


def test_mlp_conjugate_invariant_config(torch_cuda):
    """The reference's own tests/configs/mlp.yml (ConjugateInvariant ring,
    N=2^13, 8192 real slots, [29]+[26]x5 / [29,29], H=8192): the frontend's op
    stream for it runs through the C-ABI on the native CI ring (8192
    coefficients per limb, NthRoot 2^15), bit for bit against the CPU oracle's
    CI ring, and decrypts within the reference's MAE gate
    (tests/models/test_mlp.py:48)."""
    from orion_amd.backend import HipLibrary
    lib = HipLibrary().new_scheme(13, [29] + [26] * 5, [29, 29], 26, h=8192, ringtype="ConjugateInvariant", seed=5,
                                  device=0)
    assert lib.N == 1 << 13 and lib.slots == 1 << 13 and int(lib.OrionHipLogN()) == 13
    for q in lib.moduli():
        assert q % (4 << 13) == 1  # NthRoot = 4N for the CI ring
    lib.DeleteScheme()
    _replay_gpu_vs_cpu("mlp_n13_ci", seed=34)


def test_lola_conjugate_invariant_config(torch_cuda):
    """configs/lola.yml as written (ConjugateInvariant, N=2^13, 26-bit chain,
    H=8192): GPU replay bit for bit vs the oracle, MAE gate."""
    _replay_gpu_vs_cpu("lola_n13_ci", seed=35)


def test_lola_n15_matches_cpu_oracle_replay(torch_cuda):
    """BASELINE config C3 (LoLA, N=2^15): whole forward pass, bit for bit."""
    _replay_gpu_vs_cpu("lola_n15", seed=32)


@pytest.mark.parametrize("B", [6, 64])
def test_lola_n15_batch_invariance(torch_cuda, B):
    """Full-size property: a batch of B copies of one ciphertext (every kernel
    launched at batch B) gives, image by image, exactly the single-image run.
    The single-image run is bit-exact with the CPU oracle
    (test_lola_n15_matches_cpu_oracle_replay) and takes the two-pass NTT
    kernels; at B = 64 (the bench's batch) the key switches' NTTs run on the
    persistent one-limb kernels with their fused epilogues, so this carries
    the oracle's parity over to the bench configuration."""
    from orion_amd.replay import OrionStream
    st = OrionStream("lola_n15", seed=33)
    st.keygen()
    st.compile()
    lib = st.lib
    ct1 = st.encrypt_batch(st.reference_input()[None])
    x = lib.export_ciphertext(ct1)
    scale = lib.GetCiphertextScaleF(ct1)
    ref = lib.export_ciphertext(st.forward(ct1))[0]
    ctb = lib.import_ciphertext(np.repeat(x, B, axis=0), scale)
    got = lib.export_ciphertext(st.forward(ctb))
    for b in range(B):
        assert np.array_equal(got[b], ref), b
    lib.DeleteScheme()


def test_key_bundle_roundtrip(torch_cuda):
    """The device key bundle bench.py broadcasts over RCCL: export on one
    scheme, import into a fresh scheme with other seeds, keys identical."""
    torch = torch_cuda
    from orion_amd.replay import OrionStream
    st = OrionStream("lola_n13", seed=34)
    st.keygen()
    st.compile()
    lib = st.lib
    g = int(lib.GaloisElement(1))
    rlk, gk, sk = lib.export_relin_key(), lib.export_galois_key(g), lib.export_secret_key()
    n = int(lib.KeyBundleBytes(1))
    buf = torch.empty(n, dtype=torch.uint8, device="cuda")
    lib.OrionHipSynchronize()
    assert lib.lib.ExportKeyBundle(buf.data_ptr(), 1) == 0
    lib.OrionHipSynchronize()
    lib.DeleteScheme()
    st2 = OrionStream("lola_n13", lib=lib, seed=99)
    st2.compile(gen_keys=False)
    assert lib.lib.ImportKeyBundle(buf.data_ptr(), n) == 0
    lib.OrionHipSynchronize()
    assert np.array_equal(lib.export_relin_key(), rlk)
    assert np.array_equal(lib.export_galois_key(g), gk)
    assert np.array_equal(lib.export_secret_key(), sk)
    lib.DeleteScheme()


def test_resnet20_end_to_end(torch_cuda):
    """ResNet-20 (CIFAR-10) with the reference's configs/resnet.yml parameters
    (N=2^13, [60] + [30]x32, h=192): the reference frontend's op stream
    (tests/golden/resnet20_n13_*: 147 linear transforms, 138 polynomial
    evaluations for the composite-minimax ReLUs, 42 bootstraps) replayed on the
    GPU; decrypted logits vs the cleartext model (exact ReLU), the
    reference's own gate (tests/models/test_mlp.py:45-48, MAE < 0.005)."""
    from orion_amd.replay import OrionStream
    st = OrionStream("resnet20_n13", seed=3)
    st.keygen()
    st.compile()
    ct = st.encrypt_batch(st.reference_input())
    res = st.decrypt_output(st.forward(ct))[0]
    exp = st.arrays["expected_output"].reshape(-1)
    assert np.abs(res - exp).mean() < 0.005, (res, exp)
    assert np.argmax(res) == np.argmax(exp)
    st.lib.DeleteScheme()


def test_resnet20_n13_prefix_matches_cpu_oracle_replay(torch_cuda, oracle_mod):
    """the ResNet-20 N=2^13 op stream (configs/resnet.yml) from
    the input through its first Bootstrap -- 20 linear transforms, 12
    composite-minimax polynomial stages, plaintext/scalar ops with scale
    matching, the bootstrap -- replayed on the GPU and on the CPU oracle
    (oracle/replay_cpu.py, scales tracked in long double like the backend's)
    with the same keys and input ciphertext: bit for bit, same level and scale.
    The oracle's bootstrap derives its own prime chain, constants and
    diagonals; only the keys are shared."""
    from orion_amd.replay import OrionStream
    from oracle.replay_cpu import CpuStream
    st = OrionStream("resnet20_n13", seed=31)
    st.keygen()
    st.compile()
    lib = st.lib
    fwd = [e for e in st.trace["events"] if e["phase"] == "forward"]
    stop = next(i for i, e in enumerate(fwd) if e["op"] == "Bootstrap")
    ct = st.encrypt_batch(st.reference_input())
    x = lib.export_ciphertext(ct)[0]
    # first pass: every Galois key is made at the level it ends at
    lib.DeleteCiphertext(st.forward(lib.CloneCiphertext(ct), stop_after=stop))
    out_h = st.forward(lib.CloneCiphertext(ct), stop_after=stop)
    out = lib.export_ciphertext(out_h)[0]
    cpu = CpuStream("resnet20_n13")
    cpu.sk = lib.export_secret_key()
    cpu.rlk = lib.export_relin_key()
    cpu.key_source = lib.export_galois_key
    cpu.compile(keys=False, lazy=True)
    slots = fwd[stop]["args"][1]
    cfg = st.meta["config"]
    # the oracle derives the chain, constants and diagonals itself; only the keys are shared
    boot, circ = bootstrap_oracle(oracle_mod, lib, cfg["logn"], cfg["logscale"], slots, cfg.get("boot_logp") or cfg["logp"])
    cpu.bootstrappers[slots] = (boot, circ, bootstrap_keys(lib, slots))
    enc = [e for e in cpu.trace["events"] if e["phase"] == "input" and e["op"] == "Encode"][0]
    ref, lvl, scale = cpu.forward((x, x.shape[1] - 1, enc["args"][2]), stop_after=stop)
    assert lib.GetCiphertextLevel(out_h) == lvl
    assert lib.GetCiphertextScaleF(out_h) == float(scale)
    assert np.array_equal(out, ref)
    st.lib.DeleteScheme()


def test_resnet20_n16_end_to_end(torch_cuda):
    """BASELINE config C4: ResNet-20 (CIFAR-10) at N = 2^16 with
    configs/resnet.yml's chain ([60] + [30] x 32, P = [60, 60], boot LogP
    [61] x 8): the reference frontend's op stream (tests/golden/resnet20_n16_*:
    23 linear transforms of up to 900 diagonals, 57 polynomial evaluations,
    18 bootstraps at slot counts 4096/8192/16384) replayed on the GPU; the
    decrypted logits meet the reference's gate (tests/models/test_mlp.py:48,
    MAE < 0.005) with the cleartext argmax.  Rotation keys are made for the
    levels of their transforms (level-scoped keys), which is what lets the
    48-prime bootstrapping chain's key set fit in HBM."""
    from orion_amd.replay import OrionStream
    st = OrionStream("resnet20_n16", seed=3)
    st.keygen()
    st.compile()
    ct = st.encrypt_batch(st.reference_input())
    res = st.decrypt_output(st.forward(ct))[0]
    exp = st.arrays["expected_output"].reshape(-1)
    assert np.abs(res - exp).mean() < 0.005, (res, exp)
    assert np.argmax(res) == np.argmax(exp)
    st.lib.DeleteScheme()


def test_library_deferral_matches_undeferred(torch_cuda, monkeypatch):
    """The library's own rewrites behind the unchanged C-ABI (RotateNew +
    AddCiphertext + DeleteCiphertext as one key switch with the addition in
    its store; RescaleNew's result sharing the rescaled input's buffer
    copy-on-write) give exactly the result with them off (ORION_DEFER=0), on
    the op-by-op replay of the reference stream: LoLA N=2^13 at batch 5 (the
    latency kernels' scatter-add store) and N=2^15 at batch 40 (the one-pass
    kernel's)."""
    import numpy as np
    from orion_amd.replay import OrionStream
    for name, B in (("lola_n13", 5), ("lola_n15", 40)):
        outs = []
        for defer in ("0", "1"):
            monkeypatch.setenv("ORION_DEFER", defer)
            st = OrionStream(name, seed=37)
            st.keygen()
            st.compile()
            lib = st.lib
            rng = np.random.default_rng(41)
            imgs = rng.standard_normal((B,) + np.asarray(st.reference_input()).shape[1:]).astype(np.float32)
            ct = st.encrypt_batch(imgs)
            outs.append(lib.export_ciphertext(st.forward(ct)))
            lib.DeleteScheme()
        assert np.array_equal(outs[0], outs[1]), name


def test_peer_pipelines_interleaved(torch_cuda):
    """Peer pipelines (OrionHipPeerCreate / OrionHipPeerSelect): a second
    context on the scheme's chain with copies of its keys, its own stream,
    pool and handles.  Two pipelines replayed op by op in turn
    (OrionStream.forward_interleaved, their kernels concurrent on the GPU)
    give, for the same input ciphertext, exactly the single pipeline's output
    -- LoLA N=2^13 at batch 3 and N=2^15 at batch 4, also with the peer
    started 3 ops behind; a peer's handles are unknown to context 0;
    DeleteScheme removes the peers."""
    import numpy as np
    from orion_amd.replay import OrionStream
    for name, B in (("lola_n13", 3), ("lola_n15", 4)):
        st = OrionStream(name, seed=91)
        st.keygen()
        st.compile()
        st2 = OrionStream(name, peer_of=st)
        st2.compile()
        lib = st.lib
        assert lib.OrionHipPeerCount() == 2 and st2.ctx_id == 1
        rng = np.random.default_rng(92)
        imgs = rng.standard_normal((B,) + np.asarray(st.reference_input()).shape[1:]).astype(np.float32)
        ct = st.encrypt_batch(imgs)
        x, scale = lib.export_ciphertext(ct), lib.GetCiphertextScaleF(ct)
        st2.use()
        ct2 = lib.import_ciphertext(x, scale)
        st.use()
        ref = lib.export_ciphertext(st.forward(lib.CloneCiphertext(ct)))
        # phase-shifted: the peer starts 3 ops behind, its stream waiting on the
        # GPU for context 0's work so far (OrionHipStreamWaitPeer)
        ca = lib.CloneCiphertext(ct)
        st2.use()
        cb = lib.CloneCiphertext(ct2)
        outs_lag = OrionStream.forward_interleaved([(st, ca), (st2, cb)], lag=3)
        st.use()
        assert np.array_equal(lib.export_ciphertext(outs_lag[0]), ref), name
        lib.DeleteCiphertext(outs_lag[0])
        st2.use()
        assert np.array_equal(lib.export_ciphertext(outs_lag[1]), ref), name
        lib.DeleteCiphertext(outs_lag[1])
        outs = OrionStream.forward_interleaved([(st, ct), (st2, ct2)])
        st.use()
        got0 = lib.export_ciphertext(outs[0])
        st2.use()
        got1 = lib.export_ciphertext(outs[1])
        assert np.array_equal(got0, ref) and np.array_equal(got1, ref), name
        # each context's handles live in a range of their own: a peer's handle
        # passed to context 0 is unknown there, never another ciphertext
        assert outs[0] < 1 << 20 <= outs[1] < 2 << 20, (outs, name)
        st.use()
        with pytest.raises(RuntimeError, match="handle not found"):
            lib.GetCiphertextLevel(outs[1])
        # the peer decrypts with its copy of the secret
        dec = st2.decrypt_output(outs[1])
        exp = st.arrays["expected_output"].reshape(-1)
        assert dec.shape[0] == B
        st.use()
        lib.DeleteScheme()
        assert lib.OrionHipPeerCount() == 0
