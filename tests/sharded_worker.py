"""One rank of the multi-process sharded tests (tests/test_gpu_sharded.py).

Started as a child process per rank (RANK, WORLD_SIZE, MASTER_ADDR,
MASTER_PORT in the environment); every rank uses HIP device 0 and a gloo
process group, proves ONE proof with bpg_r1cs_prove_sharded (dist.sharded_prove)
and verifies it with the sharded verifier, then writes its results as JSON to
argv[2].

usage: python tests/sharded_worker.py <statement> <out.json> [ipp_tail]
  statement: config2 | config3 | fixture:<name>      (seed 4242, entropy 0..31)
           | golden:config4 | golden:config5 | golden:merkle512
             (tests/golden/fullsize.json: its seed, entropy and label, so the
             proof must equal the committed oracle proof byte for byte)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "bulletproof-gadgets_amd"), os.path.join(ROOT, "oracle")]

# merkle_tree_gadget.rs:126-131 (W1) and :475 (the hash_512 root)
W1 = bytes.fromhex("0522a64d7b931e21760cf955a15fcc793e8a52b42a56ab03afddec8beb668749")
ROOT512 = bytes.fromhex("038c137beec8e2edfb5c48cbd063f04e569139d2221a4eb7befb85aa1bf8ba40")


def statement(name):
    import workloads as W
    if name.startswith("fixture:"):
        base = os.path.join(ROOT, "tests", "golden", "resources", name.split(":", 1)[1])
        return tuple(open(base + "." + e).read() for e in ("inst", "wtns", "gadgets"))
    return W.CONFIGS[int(name[-1])]()


def golden_view(bpg, name):
    """(label, view, entropy, keep-alive) of a fullsize.json statement, built
    as tests/test_gpu_fullsize.py builds it."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))[name]
    if name == "merkle512":
        import synth as S   # the seeded ChaCha20 stream of the oracle (test infrastructure)
        rng = S.Rng(g["seed"])
        cs = bpg.GadgetCS(prover=True)
        w = int.from_bytes(W1, "big")
        variables = [cs.commit(w, rng.scalar()) for _ in range(512)]
        pattern = ("W",)
        for _ in range(9):
            pattern = ("H", pattern, pattern)
        cs.merkle_tree([(bpg.ONE, int.from_bytes(ROOT512, "big"))], [], [[(v, 1)] for v in variables],
                       bpg.pattern_str(pattern))
        ent = rng.bytes(32)
        return g, cs.view, ent, cs
    inst, wit, gad = statement(name)
    bpg.set_seed(g["seed"])
    syn = bpg.Synth(inst, wit, gad)
    return g, syn.view, bytes.fromhex(g["entropy"]), syn


def main():
    import torch.distributed as dist
    import dist as D
    import workloads as W
    name, out = sys.argv[1], sys.argv[2]
    tail = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bpg = W._bpg()
    ctx = bpg.Context(0)
    ctx.set_strategy(ipp_tail=tail)
    res = {"rank": rank}
    if name.startswith("golden:"):
        g, view, ent, keep = golden_view(bpg, name.split(":", 1)[1])
        label = g["label"].encode()
        res["golden"] = g["proof"]
    else:
        inst, wit, gad = statement(name)
        bpg.set_seed(4242)
        keep = bpg.Synth(inst, wit, gad)
        view, ent, label = keep.view, bytes(range(32)), b"sharded"
    proof, V = D.sharded_prove(ctx, label, view, ent)
    res["comb_bytes"] = ctx.setup_stats()["comb_bytes"]   # > 0: the comb-table fold ran
    # the verifier's mega-MSM split over the same ranks: per call (bpg_r1cs_verify_shard)
    # and with the circuit prepared once (bpg_verify_prepared)
    ok = D.sharded_verify(bpg, ctx, label, view, V, proof)
    prep = ctx.prepare(view, verifier=True)
    ok_prep = D.sharded_verify_prepared(bpg, prep, label, V, proof)
    bad = bytearray(proof)
    bad[1 + 8 * 32 + 3 * 32 + 5] ^= 1          # inside L_0
    bad_ok = D.sharded_verify(bpg, ctx, label, view, V, bytes(bad))
    bad_ok_prep = D.sharded_verify_prepared(bpg, prep, label, V, bytes(bad))
    res.update({"proof": proof.hex(), "V": b"".join(V).hex(), "verify": ok, "verify_prepared": ok_prep,
                "verify_tampered": bad_ok, "verify_prepared_tampered": bad_ok_prep})
    with open(out, "w") as f:
        json.dump(res, f)
    del keep
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
