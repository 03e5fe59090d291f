"""One rank of the multi-process sharded tests (tests/test_gpu_sharded.py).

Started as a child process per rank (RANK, WORLD_SIZE, MASTER_ADDR,
MASTER_PORT in the environment); every rank uses HIP device 0 and a gloo
process group, proves ONE proof with bpg_r1cs_prove_sharded (dist.sharded_prove)
and verifies it with the sharded verifier (dist.sharded_verify), then writes
its results as JSON to argv[2].

usage: python tests/sharded_worker.py <statement> <out.json>
  statement: config2 | config3 | fixture:<name>
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bulletproof-gadgets_amd")]


def statement(name):
    import workloads as W
    if name.startswith("fixture:"):
        base = os.path.join(ROOT, "tests", "golden", "resources", name.split(":", 1)[1])
        return tuple(open(base + "." + e).read() for e in ("inst", "wtns", "gadgets"))
    return W.CONFIGS[int(name[-1])]()


def main():
    import torch.distributed as dist
    import dist as D
    import workloads as W
    name, out = sys.argv[1], sys.argv[2]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bpg = W._bpg()
    inst, wit, gad = statement(name)
    bpg.set_seed(4242)
    syn = bpg.Synth(inst, wit, gad)
    ctx = bpg.Context(0)
    ent = bytes(range(32))
    proof, V = D.sharded_prove(ctx, b"sharded", syn.view, ent)
    ok = D.sharded_verify(bpg, ctx, b"sharded", syn.view, V, proof)
    bad = bytearray(proof)
    bad[1 + 8 * 32 + 3 * 32 + 5] ^= 1          # inside L_0
    bad_ok = D.sharded_verify(bpg, ctx, b"sharded", syn.view, V, bytes(bad))
    with open(out, "w") as f:
        json.dump({"rank": rank, "proof": proof.hex(), "V": b"".join(V).hex(), "verify": ok,
                   "verify_tampered": bad_ok}, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
