"""World-size-2 tests of the multi-GPU plumbing on the CPU (gloo backend):
the exchange used by the sharded verifier (all-gather of 33-byte messages,
host Ristretto point sum in libbpg) and the bench's max-over-ranks timing.
Partials are computed by the CPU oracle here (no GPU): rank r sums its slice
of one MSM; the gathered partials must add up to the oracle's full MSM, and
a verdict is an identity check over them (dist.combine_verify)."""
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
