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
