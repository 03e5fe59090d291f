"""Tests of the multi-GPU plumbing (dist.py).

CPU (gloo, world size 2): the exchange used by the sharded verifier
(all-gather of 33-byte messages, host Ristretto point sum in libbpg) and the
bench's max-over-ranks timing. Without a GPU the partials come from the CPU
oracle: rank r sums its slice of one MSM; the gathered partials must add up to
the oracle's full MSM, and a verdict is an identity check over them
(dist.combine_verify).

GPU (-m gpu): the same exchange with the product's own partials
(bpg_verify_prepared) over gloo at world size 2, and the RCCL ("nccl")
process group bench.py uses, at world size 1 (tests/dist_worker.py)."""
import os
import random
import socket
import sys

import pytest
import torch.multiprocessing as mp

from conftest import ROOT

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, out_dir):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "bulletproof-gadgets_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as tdist
    tdist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import oracle as O
        import workloads as W
        import dist as D
        bpg = W._bpg()
        L = 2**252 + 27742317777372353535851937790883648493
        rnd = random.Random(42)                    # same points/scalars on every rank
        pts = [O.from_uniform(bytes(rnd.getrandbits(8) for _ in range(64))) for _ in range(40)]
        sc = [rnd.randrange(L).to_bytes(32, "little") for _ in range(40)]
        full = O.msm(sc, pts)
        lo, hi = rank * 40 // WORLD, (rank + 1) * 40 // WORLD
        part = O.msm(sc[lo:hi], pts[lo:hi])
        msgs = D.all_gather_bytes(b"\x01" + part)
        res = {"sum_ok": bpg.point_sum([m[1:] for m in msgs]) == full,
               "order_ok": msgs[rank][1:] == part}
        # a verdict: append -full on rank 0 so that the partials cancel
        neg = O.point_mul((L - 1).to_bytes(32, "little"), full)
        part2 = O.point_add(part, neg) if rank == 0 else part
        res["accept"] = D.combine_verify(bpg, D.all_gather_bytes(b"\x01" + part2))
        res["reject_sum"] = not D.combine_verify(bpg, D.all_gather_bytes(b"\x01" + part))
        res["reject_flag"] = not D.combine_verify(bpg, D.all_gather_bytes(bytes([0 if rank == 1 else 1]) + part2))
        res["max"] = D.max_over_ranks(1.5 + rank) == 1.5 + WORLD - 1
        with open(os.path.join(out_dir, "r%d" % rank), "w") as f:
            f.write(repr(res))
    finally:
        tdist.destroy_process_group()


def test_gloo_world2_sharded_exchange(tmp_path):
    mp.spawn(_worker, args=(_free_port(), str(tmp_path)), nprocs=WORLD, join=True)
    for r in range(WORLD):
        res = eval(open(os.path.join(tmp_path, "r%d" % r)).read())
        assert all(res.values()), (r, res)


def _run_device_ranks(backend, world, tmp_path):
    import json
    import subprocess
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "dist_worker.py"), backend,
                                       str(tmp_path / ("r%d.json" % r))], env=env))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=150))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert rcs == [0] * world, rcs
    return [json.load(open(tmp_path / ("r%d.json" % r))) for r in range(world)]


@pytest.mark.gpu
def test_nccl_world1_exchange(tmp_path):
    """The RCCL process group bench.py initialises between GPUs, at world
    size 1 on cuda:0: the cuda-tensor all-gather and MAX all-reduce of
    dist.py, and verdicts through dist.sharded_verify(_prepared) and through
    two shards' product partials combined over the gather."""
    (res,) = _run_device_ranks("nccl", 1, tmp_path)
    assert res["backend"] == "nccl" and res["world"] == 1 and res["comm_device"].startswith("cuda")
    for k in ("gather_ok", "max_ok", "accept", "reject", "accept_per_call", "accept2", "reject2"):
        assert res[k] is True, (k, res)


@pytest.mark.gpu
def test_gloo_world2_product_partials(tmp_path):
    """World 2 over gloo with the PRODUCT's shard partials (bpg_verify_prepared
    on the device, one shard per rank): a valid proof's partials add up to the
    identity, a tampered proof's do not."""
    res = _run_device_ranks("gloo", 2, tmp_path)
    for r in res:
        assert r["world"] == 2
        for k in ("gather_ok", "max_ok", "accept", "reject"):
            assert r[k] is True, (k, r)
