"""GPU debugging aid (not part of the suite): run the LoLA N=2^15 forward pass
twice at batch 1 on clones of one ciphertext and report the first replayed op
whose output differs between the two runs (hash of every op's exported
output).  Run after the GPU suite's earlier modules in the same process:
  python -m pytest -q tests/test_gpu_boundary.py tests/test_gpu_ci.py \
      tests/test_gpu_ops.py -k "not batch_invariance" tools/dbg_lola_determinism.py"""
import hashlib

import numpy as np
import pytest


def _run(st, ct):
    lib = st.lib
    log = []

    def hook(ev, h):
        if isinstance(h, int) and h >= 0 and ev["op"] not in ("DeletePlaintext",):
            try:
                a = lib.export_ciphertext(h)
            except Exception:
                return
            log.append((ev["op"], hashlib.sha1(a.tobytes()).hexdigest()[:12]))

    x = lib.CloneCiphertext(ct)
    out = st.forward(x, hook=hook)
    res = lib.export_ciphertext(out)
    return log, res


@pytest.mark.gpu
def test_lola_n15_determinism():
    from orion_amd.replay import OrionStream
    st = OrionStream("lola_n15", seed=33)
    st.keygen()
    st.compile()
    ct1 = st.encrypt_batch(st.reference_input()[None])
    runs = [_run(st, ct1) for _ in range(3)]
    for r in range(1, 3):
        for i, (a, b) in enumerate(zip(runs[0][0], runs[r][0])):
            if a != b:
                print(f"run 0 vs {r}: first difference at op {i} {a[0]} ({a[1]} vs {b[1]})")
                break
        else:
            print(f"run 0 vs {r}: all {len(runs[0][0])} op outputs equal")
    assert all(np.array_equal(runs[0][1], r[1]) for r in runs[1:])
    st.lib.DeleteScheme()


@pytest.mark.gpu
def test_lola_n15_batch_invariance_repeat():
    """The suite's batch-invariance scenario repeated (REPS, default 6) in one
    process; prints which repetitions differ."""
    import os
    from orion_amd.replay import OrionStream
    bad = []
    for rep in range(int(os.environ.get("REPS", 6))):
        st = OrionStream("lola_n15", seed=33)
        st.keygen()
        st.compile()
        lib = st.lib
        ct1 = st.encrypt_batch(st.reference_input()[None])
        x = lib.export_ciphertext(ct1)
        scale = lib.GetCiphertextScaleF(ct1)
        ref = lib.export_ciphertext(st.forward(ct1))[0]
        ctb = lib.import_ciphertext(np.repeat(x, 6, axis=0), scale)
        got = lib.export_ciphertext(st.forward(ctb))
        ok = all(np.array_equal(got[b], ref) for b in range(6))
        print(f"rep {rep}: {'equal' if ok else 'DIFFERENT'} ref[0,0,0] {ref[0, 0, 0]} got[0,0,0,0] {got[0, 0, 0, 0]}")
        if not ok:
            bad.append(rep)
        lib.DeleteScheme()
    assert not bad, bad
