"""The reference's accept/reject matrix on the device (VERDICT r1
item 2): for every round-trip test of the reference crate the device proof
(bpg_r1cs_prove over the test's Gadget-API circuit) is byte-identical to the
oracle's, and the device verdict (bpg_r1cs_verify, and bpg_verify_batch over
the whole matrix of one circuit family) equals the verdict the reference
asserts. The 12 CI prove -> verify runs of the CLI binaries
(.github/workflows/integration_tests.yml:19-58) run the product's bin/prover
and bin/verifier with the reference's argv-path transcript label
(src/bin/prover.rs:17).
"""
import os
import shutil
import subprocess

import pytest

import reference_matrix as M
import synth as S
from conftest import read_fixture

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bulletproof-gadgets_amd", "bin")
CI = ["bounds_check", "equality", "inequality", "less_than", "merkle_tree", "mimc_hash", "set_membership",
      "or", "or2", "or3", "or4", "or5"]


@pytest.fixture(scope="module")
def bpg():
    import workloads
    return workloads._bpg()


@pytest.fixture(scope="module")
def ctx(bpg):
    return bpg.Context(0)


@pytest.mark.parametrize("fn,label,want,where", M.cases(), ids=[c[0] for c in M.cases()])
def test_device_matches_reference_verdict(ctx, fn, label, want, where):
    ok_oracle, o_proof, V, pf, vf, label, ent = M.oracle_verdict(fn)
    proof, dV = ctx.r1cs_prove(label, pf.view(), ent)
    assert dV == V
    assert proof == o_proof
    ok = ctx.r1cs_verify(label, vf.view(secrets=False), V, proof)
    assert ok == ok_oracle == (want == "ok"), "%s asserts is_%s" % (where, want)


def test_device_batch_verdicts(ctx, bpg):
    """The less_than family through bpg_verify_batch: one prepared verifier
    circuit per case, verdicts as the reference asserts."""
    for fn, label, want, where in M.cases():
        if "less_than" not in fn:
            continue
        _, proof, V, pf, vf, label, _ = M.oracle_verdict(fn)
        vprep = ctx.prepare(vf.view(secrets=False), verifier=True)
        assert vprep.verify_batch(label, V, [proof, proof], 2) == [want == "ok"] * 2, where


@pytest.mark.parametrize("name", CI)
def test_cli_prover_verifier(tmp_path, name):
    """cargo run --bin prover tests/resources/<name> then --bin verifier: the
    product's binaries print `true`; the transcript label is the argv path,
    so the same files under another path do not verify; with --seed the
    proof equals the oracle's for that label."""
    res = tmp_path / "tests" / "resources"
    res.mkdir(parents=True)
    for ext in ("inst", "wtns", "gadgets"):
        shutil.copy(os.path.join(ROOT, "tests", "golden", "resources", name + "." + ext), res / (name + "." + ext))
    base = "tests/resources/" + name
    run = lambda *a: subprocess.run(list(a), cwd=tmp_path, capture_output=True, text=True, timeout=120)  # noqa: E731
    p = run(os.path.join(BIN, "prover"), base, "--seed", "99")
    assert p.returncode == 0, p.stderr
    q = int(p.stdout.split()[0])
    v = run(os.path.join(BIN, "verifier"), base)
    assert v.returncode == 0 and v.stdout.strip() == "true", (v.stdout, v.stderr)
    fx = read_fixture(os.path.join(ROOT, "tests", "golden", "resources", name))
    o_proof, o_coms, flat = S.prove_statement(base.encode(), fx["inst"], fx["wtns"], fx["gadgets"], 99)
    assert (tmp_path / (base + ".proof")).read_bytes() == o_proof
    assert (tmp_path / (base + ".coms")).read_text() == o_coms
    assert q == flat.q
    # the label is the path string: ./tests/resources/<name> is another transcript
    v2 = run(os.path.join(BIN, "verifier"), "./" + base)
    assert v2.stdout.strip() == "false"
