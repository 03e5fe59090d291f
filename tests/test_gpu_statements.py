"""bpg_prove_statements (prove.rs:37-82 for many distinct statements at
once): statement k must give exactly the bytes of
`set_seed(seeds[k]); c_prove(name, *statement_k)` — the same synthesis,
commitments and proof — although its TranscriptRng stream is drawn in
lockstep with up to 7 other statements of different sizes, distinct
statements of one shape are proved up to four at a time in lockstep (their
IPP MSM jobs merged), and a statement that fails to synthesise yields None
without disturbing the others."""
import os

import pytest

from conftest import read_fixture

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bpg():
    import workloads
    return workloads._bpg()


def test_prove_statements_matches_c_prove(bpg):
    import workloads as W
    res = os.path.join(ROOT, "tests", "golden", "resources")
    sts = []
    for name in ("bounds_check", "mimc_hash", "or3", "set_membership", "merkle_tree", "less_than", "example"):
        fx = read_fixture(os.path.join(res, name))
        sts.append((fx["inst"], fx["wtns"], fx["gadgets"]))
    sts += [W.config2(), W.config3(), W.config2(2002)]
    bad = ("I0 = 0x11\n", "W0 = 0x43\n", "FOO W0\n")        # unknown gadget
    sts.insert(4, bad)
    seeds = [7000 + 13 * k for k in range(len(sts))]
    out = bpg.prove_statements("stmts", sts, threads=6, seeds=seeds)
    assert len(out) == len(sts)
    for k, (st, seed) in enumerate(zip(sts, seeds)):
        if st is bad:
            assert out[k] is None
            continue
        bpg.set_seed(seed)
        want = bpg.prove("stmts", *st)
        assert out[k] is not None, k
        assert out[k][1] == want[1], "coms of statement %d" % k
        assert out[k][0] == want[0], "proof of statement %d" % k
        assert bpg.verify("stmts", st[0], out[k][0], out[k][1], st[2])
    # per-stage counters of the call (bpg_last_statements_stats), and the HBM
    # budget sized from the first prepared statement (statement buffers are
    # recycled across the call's statements of different sizes above)
    st = bpg.last_statements_stats()
    assert st["workers"] == 6 and st["consumers"] == 3
    assert st["est_gb_per_statement"] > 0 and st["hbm_limit"] >= st["consumers"] + 1
    assert st["limit"] <= 4 * 6 + 8 + 2 * 3
    assert st["bound_stage"] in ("cpu workers (synthesis + prepare + rng)", "device consumers")
    assert st["synth_ms"] > 0 and st["prove_ms"] > 0 and st["rng_ms"] > 0


def test_prove_statements_same_shape_lockstep(bpg):
    """Distinct statements of one shape (config 2 with different seeds: other
    witnesses, Merkle roots and set elements, the same n, m, N) are proved in
    lockstep by the device threads; each proof still equals its own c_prove."""
    import workloads as W
    sts = [W.config2(3100 + k) for k in range(9)]
    seeds = [900 + k for k in range(len(sts))]
    out = bpg.prove_statements("same", sts, threads=4, seeds=seeds)
    for k, (st, seed) in enumerate(zip(sts, seeds)):
        bpg.set_seed(seed)
        want = bpg.prove("same", *st)
        assert out[k] == want, k
    assert len(set(o[0] for o in out)) == len(sts)
