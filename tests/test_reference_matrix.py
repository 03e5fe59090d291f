"""CPU: the oracle's accept/reject verdicts on every round-trip test of the
reference crate equal the verdicts the reference asserts (27 is_ok + 11
is_err, tests/golden/reference_cases.json, extracted from the reference's own
test sources). This pins the oracle's protocol at the third-party boundary,
where no reference proof bytes exist. The device verdicts are in
test_gpu_reference_matrix.py.
"""
import json
import os

import pytest

import reference_matrix as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_extracted_matrix_is_complete():
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_cases.json")))
    tests = [t for v in d.values() for t in v["tests"]]
    assert len(tests) == 38
    assert sum(t["verdict"] == "ok" for t in tests) == 27
    assert sum(t["verdict"] == "err" for t in tests) == 11
    assert {t["fn"] for t in tests if t["ignored"]} == {"test_merkle_tree_gadget_512"}


@pytest.mark.parametrize("fn,label,want,where", M.cases(), ids=[c[0] for c in M.cases()])
def test_oracle_verdict_matches_reference(fn, label, want, where):
    ok = M.oracle_verdict(fn)[0]
    assert ok == (want == "ok"), "%s asserts is_%s" % (where, want)
