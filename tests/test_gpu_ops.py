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


@pytest.mark.parametrize("B", [6, 32, 64])
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


@pytest.mark.parametrize("name", ["lola_n13", "lola_n13_ci", "mlp_n14"])
def test_thread_pipelines_small(torch_cuda, name):
    """Thread-affine pipelines (OrionHipThreadPipelines): two frontend threads
    each run the unchanged op stream's forward() (one compiled stream: the
    scheme's keys and transforms) on a ciphertext they imported themselves; the
    library binds each thread to a context of its own (own stream, pool,
    handle range), and each output equals the scheme thread's single run bit
    for bit -- at batch 3, LoLA N=2^13 on the Standard and the
    ConjugateInvariant ring (configs/lola.yml) and the MLP at N=2^14
    (BASELINE C2).  Handles are unique across contexts:
    the main thread reads and deletes the pipelines' outputs; an in-place op
    on another context's ciphertext is refused; DeleteScheme removes the
    pipelines."""
    import numpy as np
    from orion_amd.replay import OrionStream, Pipelines
    st = OrionStream(name, seed=91)
    st.keygen()
    st.compile()
    lib = st.lib
    B = 3
    rng = np.random.default_rng(92)
    imgs = rng.standard_normal((B,) + np.asarray(st.reference_input()).shape[1:]).astype(np.float32)
    ct = st.encrypt_batch(imgs)
    x, scale = lib.export_ciphertext(ct), lib.GetCiphertextScaleF(ct)
    ref = lib.export_ciphertext(st.forward(lib.CloneCiphertext(ct)))
    pipes = Pipelines(lib, 2, device=0)
    try:
        assert sorted(pipes.contexts) == [1, 2] and lib.OrionHipPeerCount() == 3
        assert lib.OrionHipCurrentPipeline() == 0  # the scheme's thread keeps the scheme's context
        cts = pipes.run([lambda: lib.import_ciphertext(x, scale)] * 2)
        for i, c in enumerate(cts):
            assert c >> 20 == pipes.contexts[i]
        for _ in range(2):  # twice: the second pass reuses each pipeline's pooled buffers
            outs = pipes.run([(lambda c=c: st.forward(c)) for c in cts])
            for o in outs:
                assert np.array_equal(lib.export_ciphertext(o), ref)  # read from the main thread
                lib.DeleteCiphertext(o)  # deleted on its own context
        # a pipeline captures its pass into a hipGraph (the scheme's compiled
        # transforms held by the graph); any thread launches it on the
        # pipeline's stream (graph ids route like handles)
        gid, gout = pipes.run_one(0, lambda: st.capture(cts[0]))
        assert gid >> 20 == pipes.contexts[0]
        lib.OrionHipGraphLaunch(gid)
        lib.OrionHipSynchronize()
        assert np.array_equal(lib.export_ciphertext(gout), ref)
        lib.OrionHipGraphDestroy(gid)
        lib.DeleteCiphertext(gout)
        with pytest.raises(RuntimeError, match="changed only by the context"):
            lib.Rescale(cts[0])
        dec = pipes.run_one(1, lambda: st.decrypt_output(cts[1]))  # the pipelines share the scheme's secret
        assert dec.shape[0] == B
    finally:
        pipes.close()
    lib.DeleteScheme()
    assert lib.OrionHipPeerCount() == 0


def test_thread_pipelines_lola_n15_timed_config(torch_cuda):
    """The bench's timed configuration, bit for bit: LoLA N=2^15, two frontend
    threads with 32 images each on their own pipeline contexts (bench.py
    --pipelines 2, batch 64).  64 different images are encrypted once; every
    image's output from the threads equals the single-image run of that
    image's ciphertext on the scheme's context (the batch-1 path that
    test_lola_n15_matches_cpu_oracle_replay checks against the CPU oracle)."""
    import numpy as np
    from orion_amd.replay import OrionStream, Pipelines
    st = OrionStream("lola_n15", seed=33)
    st.keygen()
    st.compile()
    lib = st.lib
    rng = np.random.default_rng(5)
    imgs = rng.standard_normal((64,) + np.asarray(st.reference_input()).shape[1:]).astype(np.float32)
    imgs[0] = np.asarray(st.reference_input()).reshape(imgs.shape[1:])
    ct = st.encrypt_batch(imgs)
    x, scale = lib.export_ciphertext(ct), lib.GetCiphertextScaleF(ct)
    lib.DeleteCiphertext(ct)
    pipes = Pipelines(lib, 2, device=0)
    try:
        cts = pipes.run([(lambda i=i: lib.import_ciphertext(x[32 * i:32 * (i + 1)], scale)) for i in range(2)])
        pipes.run([(lambda c=c: lib.DeleteCiphertext(st.forward(lib.CloneCiphertext(c)))) for c in cts])  # warm
        outs = pipes.run([(lambda c=c: st.forward(c)) for c in cts])
        got = np.concatenate([lib.export_ciphertext(o) for o in outs])
    finally:
        pipes.close()
    assert got.shape[0] == 64
    for b in range(64):
        one = lib.import_ciphertext(x[b:b + 1], scale)
        assert np.array_equal(lib.export_ciphertext(st.forward(one))[0], got[b]), b
    res = st.decrypt_output(lib.import_ciphertext(got[:1], lib.GetCiphertextScaleF(outs[0])))[0]
    assert np.abs(res - st.arrays["expected_output"].reshape(-1)).mean() < 0.005
    lib.DeleteScheme()


def test_pool_cap_forces_trim_and_retry(torch_cuda):
    """The failed-allocation path (the a6cfbba fix): under a
    pool byte cap (OrionHipPoolCap, = ORION_POOL_CAP_BYTES) an allocation past
    the cap releases every pool's cache and retries once.  A chain whose
    buffer sizes are new, run with the cap at the bytes held (cache full of
    other sizes), forces that trim, leaves no stale HIP error for the next
    call, and gives the uncapped run's output bit for bit; a cap below the
    live bytes fails the call with a clear error, and the scheme works again
    once the cap is lifted."""
    import numpy as np
    from orion_amd.backend import HipLibrary
    lib = HipLibrary().new_scheme(13, [55, 40, 40, 40, 40, 40], [60, 60], 40, h=192, seed=7, device=0)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    lib.AddRotationKey(5)
    rng = np.random.default_rng(0)

    def enc(B):
        return lib.Encrypt(lib.encode_batch(rng.standard_normal((B, 4096)).astype(np.float32), 5, 1 << 40))

    def chain(ct):
        a = lib.MulRelinCiphertextNew(ct, ct)
        b = lib.RotateNew(a, 5)
        lib.Rescale(b)
        c = lib.AddCiphertextNew(b, b)
        out = lib.export_ciphertext(c)
        for h in (a, b, c):
            lib.DeleteCiphertext(h)
        return out

    ct16, ct32 = enc(16), enc(32)
    chain(enc(4))
    # the cache fills with buffers of a size the chain at batch 16 never takes
    junk = [lib.encode_batch(np.zeros((64, 4096), np.float32), 5, 1 << 40) for _ in range(16)]
    for h in junk:
        lib.DeletePlaintext(h)
    st1 = lib.pool_stats()
    live = st1["held_bytes"] - st1["cached_bytes"]
    assert st1["cached_bytes"] > 300e6, st1
    prev = lib.pool_cap(st1["held_bytes"])
    try:
        got = chain(ct16)  # its first new-size allocation is past the cap: trim, retry
        st2 = lib.pool_stats()
        assert st2["trims"] > st1["trims"], (st1, st2)
        assert st2["held_bytes"] <= st1["held_bytes"], (st1, st2)
        assert lib.GetCiphertextLevel(ct16) == 5  # the next call sees no stale error
        lib.pool_cap(live * 0.5)
        with pytest.raises(RuntimeError, match="device memory exhausted"):
            chain(ct32)
        assert lib.GetCiphertextLevel(ct32) == 5
    finally:
        lib.pool_cap(prev)
    assert np.array_equal(chain(ct16), got)  # uncapped: the same bits
    chain(ct32)
    lib.DeleteScheme()


def test_deferred_rotation_failure_poisons(torch_cuda):
    """a deferred rotate-and-add whose key switch fails when it runs
    (DeleteCiphertext of the rotation, here an allocation past the pool cap)
    reports the failure, deletes the rotation's handle, and poisons the
    ciphertext the AddCiphertext had reported as updated: every later use of
    it fails loudly instead of reading a buffer that was never written."""
    import numpy as np
    from orion_amd.backend import HipLibrary
    lib = HipLibrary().new_scheme(13, [55, 40, 40, 40, 40, 40], [60, 60], 40, h=192, seed=7, device=0)
    lib.GenerateSecretKey()
    lib.GeneratePublicKey()
    lib.GenerateRelinearizationKey()
    lib.AddRotationKey(1)
    vals = np.random.default_rng(1).standard_normal((2, 4096)).astype(np.float32)
    x = lib.Encrypt(lib.encode_batch(vals, 5, 1 << 40))
    live0 = lib.GetLiveCiphertexts()
    r = lib.RotateNew(x, 1)
    assert lib.AddCiphertext(x, r) == x
    st = lib.pool_stats()
    lib.pool_cap(st["held_bytes"] - st["cached_bytes"])  # nothing new fits
    try:
        with pytest.raises(RuntimeError, match="device memory exhausted"):
            lib.DeleteCiphertext(r)
    finally:
        lib.pool_cap(0)
    assert lib.GetLiveCiphertexts() == live0  # r is gone
    with pytest.raises(RuntimeError, match="deferred rotation by 1 failed"):
        lib.GetCiphertextLevel(x)
    lib.DeleteCiphertext(x)
    y = lib.Encrypt(lib.encode_batch(vals, 5, 1 << 40))  # the scheme still works
    assert lib.GetCiphertextLevel(lib.RotateNew(y, 1)) == 5
    lib.DeleteScheme()


def test_thread_pipeline_bootstrap_and_polynomials(torch_cuda):
    """A pipeline thread runs the ResNet-20 N=2^13 op stream (configs/resnet.yml)
    through its first Bootstrap: linear transforms, composite-minimax
    polynomial ReLUs (the scheme's compiled polynomials read from the
    pipeline) and the bootstrap itself, which a pipeline runs with the
    scheme's bootstrapper on the scheme's stream.  The output equals the
    scheme thread's run of the same ciphertext bit for bit, same level and
    scale."""
    import numpy as np
    from orion_amd.replay import OrionStream, Pipelines
    st = OrionStream("resnet20_n13", seed=31)
    st.keygen()
    st.compile()
    lib = st.lib
    fwd = [e for e in st.trace["events"] if e["phase"] == "forward"]
    stop = next(i for i, e in enumerate(fwd) if e["op"] == "Bootstrap")
    ct = st.encrypt_batch(st.reference_input())
    x, scale = lib.export_ciphertext(ct), lib.GetCiphertextScaleF(ct)
    lib.DeleteCiphertext(st.forward(lib.CloneCiphertext(ct), stop_after=stop))  # keys made at their levels
    ref_h = st.forward(lib.CloneCiphertext(ct), stop_after=stop)
    ref = lib.export_ciphertext(ref_h)
    pipes = Pipelines(lib, 1, device=0)
    try:
        out_h = pipes.run_one(0, lambda: st.forward(lib.import_ciphertext(x, scale), stop_after=stop))
        assert out_h >> 20 == pipes.contexts[0] >= 1
        assert lib.GetCiphertextLevel(out_h) == lib.GetCiphertextLevel(ref_h)
        assert lib.GetCiphertextScaleF(out_h) == lib.GetCiphertextScaleF(ref_h)
        assert np.array_equal(lib.export_ciphertext(out_h), ref)
    finally:
        pipes.close()
    lib.DeleteScheme()


def test_thread_pipelines_stress_cross_context(torch_cuda):
    """Four frontend threads on their own pipeline contexts hammer the C-ABI at
    once (the LoLA N=2^13 op stream -- linear transforms, rotate-and-adds,
    mul_relin, rescales -- then mul_relin + rotation on its output), each
    also reading the other threads' ciphertexts (AddCiphertextNew across
    contexts, ordered after the owner's queued work) and deleting handles
    another thread made (routed to the owner's context).  Every result equals the one computed by the scheme thread
    alone; no handle leaks; the thread-local last error of one thread is not
    seen by another."""
    import numpy as np
    from orion_amd.replay import OrionStream, Pipelines
    st = OrionStream("lola_n13", seed=55)
    st.keygen()
    st.compile()
    lib = st.lib
    lib.AddRotationKey(7)
    rng = np.random.default_rng(56)
    imgs = rng.standard_normal((8,) + np.asarray(st.reference_input()).shape[1:]).astype(np.float32)
    ct = st.encrypt_batch(imgs)
    x, scale = lib.export_ciphertext(ct), lib.GetCiphertextScaleF(ct)
    shards = [x[2 * i:2 * i + 2] for i in range(4)]

    def chain(h):
        out = st.forward(h)
        lib.DeleteCiphertext(h)
        sq = lib.MulRelinCiphertextNew(out, out)  # (the stream ends at level 0: no rescale)
        r = lib.RotateNew(sq, 7)
        res = lib.export_ciphertext(r)
        for k in (out, sq, r):
            lib.DeleteCiphertext(k)
        return res

    ref = [chain(lib.import_ciphertext(s, scale)) for s in shards]
    live0 = set(lib.GetLiveCiphertexts())
    pipes = Pipelines(lib, 4, device=0)
    try:
        ins = pipes.run([(lambda s=s: lib.import_ciphertext(s, scale)) for s in shards])
        for rep in range(3):
            outs = pipes.run([(lambda h=h: chain(lib.CloneCiphertext(h))) for h in ins])
            for i in range(4):
                assert np.array_equal(outs[i], ref[i]), (rep, i)
        # cross-context reads: thread i adds thread (i+1)'s input into a new ciphertext of its own
        sums = pipes.run([(lambda i=i: lib.AddCiphertextNew(ins[i], ins[(i + 1) % 4])) for i in range(4)])
        for i in range(4):
            got = lib.export_ciphertext(sums[i])
            qs = np.array(lib.moduli()[:got.shape[2]], dtype=np.uint64)[None, None, :, None]
            a = shards[i].astype(object)
            b = shards[(i + 1) % 4].astype(object)
            assert np.array_equal(got, ((a + b) % qs.astype(object)).astype(np.uint64)), i
        # an in-place op on another thread's ciphertext is refused; each
        # thread's error stays its own
        errs = pipes.run([(lambda i=i: _try(lambda: lib.Rescale(ins[(i + 1) % 4]))) for i in range(4)])
        assert all("changed only by the context" in e for e in errs), errs
        assert lib.lib.OrionHipLastError() == b""
        # deletes from other threads go to the owner's context
        pipes.run([(lambda i=i: lib.DeleteCiphertext(sums[(i + 2) % 4])) for i in range(4)])
        pipes.run([(lambda i=i: lib.DeleteCiphertext(ins[(i + 3) % 4])) for i in range(4)])
        left = pipes.run([lambda: lib.GetLiveCiphertexts()] * 4)
        assert all(len(v) == 0 for v in left), left
    finally:
        pipes.close()
    assert set(lib.GetLiveCiphertexts()) == live0
    lib.DeleteScheme()


def _try(fn):
    try:
        fn()
    except RuntimeError as e:
        return str(e)
    return ""
