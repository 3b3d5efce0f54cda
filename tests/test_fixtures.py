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


@pytest.mark.parametrize("name,pairs", [("lola_n15", 10), ("lola_n13", "all"), ("mlp_n13", None), ("mlp_n14", None),
                                        ("resnet20_n13", None)])
def test_rotate_add_pairs(name, pairs):
    """The replay's RotateNew + AddCiphertext fusion (OrionHipRotateAdd) takes
    exactly the pairs x += Rotate(x, k) whose rotation nothing else reads:
    LoLA's rotate-and-sum steps (all of its RotateNew).  Every taken pair is adjacent, adds into
    the rotation's own input, and the rotation's handle is not read again
    before it is redefined or deleted."""
    from orion_amd.replay import rotate_add_pairs, _CT_OPS
    t, _ = load(name)
    ev = t["events"]
    got = rotate_add_pairs(ev, t["meta"].get("output_ids", []))
    if pairs == "all":
        pairs = sum(e["phase"] == "forward" and e["op"] == "RotateNew" for e in ev)
    if pairs is not None:
        assert len(got) == pairs
    for a, b in got.items():
        r, s = ev[a], ev[b]
        assert r["op"] == "RotateNew" and s["op"] == "AddCiphertext"
        assert s["args"] == [r["args"][0], r["ret"]] and s["ret"] == r["args"][0]
        for e in ev[b + 1:]:
            if e.get("ret") == r["ret"] or (e["op"] == "DeleteCiphertext" and e["args"][0] == r["ret"]):
                break
            kinds = _CT_OPS.get(e["op"], ())
            assert not any(k == "ct" and v == r["ret"] for k, v in zip(kinds, e["args"]))
    # a rotation read again later is never fused
    x = [{"phase": "forward", "op": "RotateNew", "args": [2, 4], "ret": 1},
         {"phase": "forward", "op": "AddCiphertext", "args": [2, 1], "ret": 2},
         {"phase": "forward", "op": "AddCiphertext", "args": [3, 1], "ret": 3}]
    assert rotate_add_pairs(x) == {}
    assert rotate_add_pairs(x[:2]) == {0: 1}


@pytest.mark.parametrize("name", ["lola_n15", "lola_n13", "mlp_n13", "mlp_n14", "resnet20_n13"])
def test_rescale_aliases(name):
    """The replay runs RescaleNew(x) -> y as an in-place Rescale(x) named y
    only when nothing reads x afterwards (LoLA: all three)."""
    from orion_amd.replay import rescale_aliases, _CT_OPS
    t, _ = load(name)
    ev = t["events"]
    got = rescale_aliases(ev, t["meta"].get("output_ids", []))
    if name.startswith("lola"):
        assert len(got) == sum(e["phase"] == "forward" and e["op"] == "RescaleNew" for e in ev)
    for i in got:
        x = ev[i]["args"][0]
        for e in ev[i + 1:]:
            if e.get("ret") == x or (e["op"] == "DeleteCiphertext" and e["args"][0] == x):
                break
            kinds = _CT_OPS.get(e["op"], ())
            assert not any(k == "ct" and v == x for k, v in zip(kinds, e["args"]))
