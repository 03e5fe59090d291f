"""One rank of the device-backed torch.distributed tests in tests/test_dist.py.

usage: python tests/dist_worker.py <backend> <out.json>   (RANK, WORLD_SIZE,
MASTER_ADDR, MASTER_PORT in the environment; device 0 for every rank)

backend nccl (world 1): the RCCL process group bench.py uses between GPUs,
  bound to cuda:0 — dist.all_gather_bytes / max_over_ranks move cuda tensors,
  and a config-2 proof is verified through dist.sharded_verify(_prepared) and
  through two shards of the mega-MSM whose product partials are combined by
  dist.combine_verify.
backend gloo (world 2): each rank computes ITS shard's partial with the
  product (bpg_verify_prepared on the device) and the ranks exchange the
  33-byte messages over gloo: valid iff the partials add to the identity.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bulletproof-gadgets_amd")]


def main():
    import torch
    import torch.distributed as tdist
    import dist as D
    import workloads as W
    backend, out = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if backend == "nccl":
        torch.cuda.set_device(0)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        tdist.init_process_group("gloo")
    bpg = W._bpg()
    res = {"rank": rank, "backend": tdist.get_backend(), "world": tdist.get_world_size(),
           "comm_device": str(D.comm_device())}
    res["gather_ok"] = D.all_gather_bytes(bytes([rank, 7, 9])) == [bytes([r, 7, 9]) for r in range(world)]
    res["max_ok"] = D.max_over_ranks(1.5 + rank) == 1.5 + world - 1
    bpg.set_seed(77)
    syn = bpg.Synth(*W.config2())
    ctx = bpg.Context(0)
    proof, V = ctx.r1cs_prove(b"dist", syn.view, bytes(32))
    bad = bytearray(proof)
    bad[-40] ^= 1
    bad = bytes(bad)
    prep = ctx.prepare(syn.view, verifier=True)
    res["accept"] = D.sharded_verify_prepared(bpg, prep, b"dist", V, proof)
    res["reject"] = not D.sharded_verify_prepared(bpg, prep, b"dist", V, bad)
    if world == 1:
        res["accept_per_call"] = D.sharded_verify(bpg, ctx, b"dist", syn.view, V, proof)
        # the world > 1 exchange on one rank: two shards' product partials
        for tag, p in (("accept2", proof), ("reject2", bad)):
            msgs = []
            for s in range(2):
                ok, part = prep.verify_one(b"dist", V, p, shard=s, nshards=2)
                msgs.append(bytes([1 if ok else 0]) + part)
            msgs = [D.all_gather_bytes(m)[0] for m in msgs]
            v = D.combine_verify(bpg, msgs)
            res[tag] = v if tag == "accept2" else not v
    with open(out, "w") as f:
        json.dump(res, f)
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
