"""Multi-GPU paths of SURVEY §8e exercised with several processes sharing
device 0 over a gloo process group (the code path is the one RCCL drives
across GPUs: one process per rank, partial sums exchanged by all-gather).

* bpg_r1cs_prove_sharded: ONE proof split over `world` ranks (cyclic lane
  layout) must be byte-identical, on every rank, to the single-process
  proof (bpg_r1cs_prove) and to the CPU oracle's;
* at BASELINE's full sizes (config 4 = 2^18 at 2, 4 and 8 ranks; config 5
  = 2^20 at 2, 4 and 8 ranks, the 8-GPU split the north_star names; the
  reference's merkle512 circuit, merkle_tree_gadget.rs:528, = 2^20 at 2 and
  8 ranks) every rank's proof must equal the committed oracle proof of
  tests/golden/fullsize.json, with the comb tables and the round-triple folds
  of the one-GPU default running on every rank's slice (prove.rs:78-79);
* the sharded verifier across processes, per call (bpg_r1cs_verify_shard)
  and over a circuit prepared once (bpg_verify_prepared): the product's
  partials of a valid proof add up to the identity, a tampered proof's do not.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

import synth as S
from conftest import read_fixture

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bpg():
    import workloads
    return workloads._bpg()


@pytest.fixture(scope="module")
def trimmed(bpg):
    """Tables this (pytest) process cached for earlier tests would leave the
    rank processes too little HBM for theirs: release them."""
    bpg.Context(0).trim()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_ranks(name, world, tmp_path, tail=None, timeout=100):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        args = [sys.executable, os.path.join(ROOT, "tests", "sharded_worker.py"), name,
                str(tmp_path / ("r%d.json" % r))] + ([str(tail)] if tail is not None else [])
        procs.append(subprocess.Popen(args, env=env))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=timeout))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert rcs == [0] * world, rcs
    return [json.load(open(tmp_path / ("r%d.json" % r))) for r in range(world)]


def single(bpg, name, tail=-1):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import sharded_worker as SW
    inst, wit, gad = SW.statement(name)
    bpg.set_seed(4242)
    syn = bpg.Synth(inst, wit, gad)
    ctx = bpg.Context(0)
    ctx.set_strategy(ipp_tail=tail)
    proof, V = ctx.r1cs_prove(b"sharded", syn.view, bytes(range(32)))
    return proof, b"".join(V), (inst, wit, gad)


def check_ranks(res):
    for r in res:
        assert r["verify"] is True and r["verify_prepared"] is True, "rank %d" % r["rank"]
        assert r["verify_tampered"] is False and r["verify_prepared_tampered"] is False, "rank %d" % r["rank"]


@pytest.mark.parametrize("name,world", [("config2", 2), ("fixture:or5", 2), ("config2", 4), ("config3", 2),
                                        ("config3", 8)])
def test_sharded_prove_bit_exact(bpg, tmp_path, name, world):
    ref_proof, ref_V, (inst, wit, gad) = single(bpg, name)
    res = run_ranks(name, world, tmp_path)
    check_ranks(res)
    for r in res:
        assert r["proof"] == ref_proof.hex(), "rank %d" % r["rank"]
        assert r["V"] == ref_V.hex()
    if name == "config2":
        # and the CPU oracle's bytes (same statement, same blindings)
        import oracle as O
        st = S.synthesize_prover(inst, wit, gad, 4242)
        o_proof, _ = O.r1cs_prove(b"sharded", st.cs.to_flat(), bytes(range(32)))
        assert ref_proof == o_proof


@pytest.mark.parametrize("name,world,tail", [("config3", 2, 0), ("config2", 4, 2), ("config3", 8, 3)])
def test_sharded_prove_small_ipp_tail(bpg, tmp_path, name, world, tail):
    """an IPP tail threshold below the last materialised level
    (0, 1, or 2-3 under an even lg Nl: config 2 at 4 ranks has Nl = 2^8) no
    longer ends the sharded prover outside the tail; its bytes equal the
    one-GPU proof under the same threshold."""
    ref_proof, _, _ = single(bpg, name, tail)
    res = run_ranks(name, world, tmp_path, tail)
    check_ranks(res)
    for r in res:
        assert r["proof"] == ref_proof.hex(), "rank %d" % r["rank"]


@pytest.mark.parametrize("name,world", [("config4", 2), ("config4", 4), ("config4", 8), ("config5", 2),
                                        ("config5", 4), ("config5", 8), ("merkle512", 2), ("merkle512", 8)])
def test_sharded_prove_fullsize_golden(bpg, trimmed, tmp_path, name, world):
    """BASELINE config 4 (Pippenger MSM sharded over 1/2/4/8 GPUs) and the
    2^20 statements split over up to 8 ranks: every rank's proof equals the
    committed oracle proof."""
    res = run_ranks("golden:" + name, world, tmp_path, timeout=300)
    check_ranks(res)
    for r in res:
        assert r["proof"] == r["golden"], "rank %d" % r["rank"]
        assert r["comb_bytes"] > 0, "rank %d proved without comb tables" % r["rank"]


def test_sharded_prove_rejects_small_circuit(bpg):
    """N < 8 * world is refused (the local rounds must end in the IPP tail):
    bounds_check has n = 1440, N = 2048 < 8 * 512."""
    fx = read_fixture(os.path.join(ROOT, "tests", "golden", "resources", "bounds_check"))
    bpg.set_seed(1)
    syn = bpg.Synth(fx["inst"], fx["wtns"], fx["gadgets"])
    with pytest.raises(bpg.BpgError):
        bpg.Context(0).r1cs_prove_sharded(b"x", syn.view, bytes(32), 0, 512, lambda p: [p] * 512)
    with pytest.raises(bpg.BpgError):
        bpg.Context(0).r1cs_prove_sharded(b"x", syn.view, bytes(32), 0, 3, lambda p: [p] * 3)   # not a power of 2
