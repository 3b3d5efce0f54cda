"""CPU tests of the op-stream fixtures recorded from the reference frontend
(tools/gen_fixtures.py): they must describe exactly the workload SURVEY.md §3.4
/ Appendix B measured, so the GPU bench and the parity tests replay the real
reference call sequence."""
import json
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, f"{name}_trace.json")) as f:
        t = json.load(f)
    a = np.load(os.path.join(GOLD, f"{name}_arrays.npz"), allow_pickle=False)
    return t, a


def fwd_counts(t):
    c = {}
    for e in t["events"]:
        if e["phase"] == "forward":
            c[e["op"]] = c.get(e["op"], 0) + 1
    return c


def test_lola_n15_matches_survey():
    t, a = load("lola_n15")
    m = t["meta"]
    assert m["config"]["logn"] == 15 and m["input_level"] == 5
    lts = [e for e in t["events"] if e["op"] == "GenerateLinearTransform"]
    assert [len(e["args"][0]) for e in lts] == [13, 128, 109]
    assert lts[0]["args"][0] == [0, 1, 27, 28, 29, 1264, 1265, 1292, 1293, 2019, 2020, 2021, 2047]
    assert lts[1]["args"][0] == list(range(128))
    assert [e["args"][2] for e in lts] == [5, 3, 1]
    c = fwd_counts(t)
    assert c["EvaluateLinearTransform"] == 3 and c["RotateNew"] == 10
    assert c["MulRelinCiphertextNew"] == 2 and c["RescaleNew"] == 3 and c["Rescale"] == 2
    assert c["AddPlaintext"] == 3
    for e in lts:
        assert a[e["arrays"] + "_diags"].shape == (len(e["args"][0]), 1 << 14)
    assert a["expected_output"].shape == (1, 10)


@pytest.mark.parametrize("name", ["lola_n13", "lola_n15", "mlp_n13", "mlp_n14"])
def test_fixture_integrity(name):
    t, a = load(name)
    for e in t["events"]:
        if "arrays" in e:
            keys = [k for k in a.files if k.startswith(e["arrays"] + "_")]
            assert keys, e
    assert "input" in a.files and "expected_output" in a.files
    ops = set(e["op"] for e in t["events"] if e["phase"] == "forward")
    from orion_amd.replay import _CT_OPS
    assert ops <= set(_CT_OPS) | {"Decrypt", "Decode", "DeletePlaintext", "DeleteCiphertext",
                                  "SetCiphertextScale"}


# C-ABI calls that leave a deferred rotation pending (backend.hip defer_keeps)
_DEFER_KEEPS = {"AddCiphertext", "DeleteCiphertext", "DeletePlaintext", "GetCiphertextScale", "GetCiphertextScaleF",
                "GetCiphertextLevel", "GetCiphertextSlots", "GetCiphertextDegree", "GetCiphertextBatch",
                "GetPlaintextScale", "GetPlaintextLevel", "GetPlaintextSlots", "GetPlaintextBatch",
                "GetLiveCiphertexts", "GetLivePlaintexts", "GetModuliChain", "GaloisElement"}


def deferred_rotations(events):
    """Model of the library's deferral (backend.hip Context::Deferred) over a
    stream of C-ABI calls: (rotate-and-adds fused in the key switch's store,
    rotations dropped unread, rotations run on their own)."""
    fused = dropped = plain = 0
    st = None  # (kind, x, r)
    for e in events:
        op, args = e["op"], e["args"]
        if st is not None:
            kind, x, r = st
            if op == "AddCiphertext" and kind == 1 and args == [x, r]:
                st = (2, x, r)
                continue
            if op == "DeleteCiphertext" and args[0] == r:
                fused += kind == 2
                dropped += kind == 1
                st = None
                continue
            if op not in _DEFER_KEEPS or (op == "DeleteCiphertext" and args[0] == x) or op == "AddCiphertext":
                plain += 1
                st = None
        if op == "RotateNew":
            st = (1, args[0], e["ret"])
    return fused, dropped, plain + (st is not None)


@pytest.mark.parametrize("name,fused", [("lola_n15", 10), ("lola_n13", "all"), ("mlp_n13", None),
                                        ("mlp_n14", None), ("resnet20_n13", None)])
def test_reference_stream_hits_deferred_rotate_add(name, fused):
    """The frontend's own calls (the recorded stream as the fork issues it,
    debug Decrypt/Decode included) reach the library's deferred rotate-and-add
    for every `out += out.roll(k)` of LoLA (linear.py:72-73): RotateNew,
    AddCiphertext into its source, DeleteCiphertext of the rotation -- so the
    op-by-op replay the bench times runs them as one key switch each."""
    t, _ = load(name)
    ev = [e for e in t["events"] if e["phase"] == "forward"]
    f, d, p = deferred_rotations(ev)
    n_rot = sum(e["op"] == "RotateNew" for e in ev)
    assert f + d + p == n_rot
    if fused == "all":
        fused = n_rot
    if fused is not None:
        assert f == fused and p == 0
    # a rotation read again, or its source written first, runs on its own
    x = [{"op": "RotateNew", "args": [2, 4], "ret": 1}, {"op": "AddCiphertext", "args": [2, 1], "ret": 2},
         {"op": "AddCiphertext", "args": [3, 1], "ret": 3}, {"op": "DeleteCiphertext", "args": [1], "ret": None}]
    assert deferred_rotations(x) == (0, 0, 1)
    assert deferred_rotations(x[:2] + x[3:]) == (1, 0, 0)
    assert deferred_rotations([x[0], x[3]]) == (0, 1, 0)
