"""Child process of tests/test_gpu_robustness.py (a fresh device context per
run). usage: robust_worker.py cache <dir> | concurrent"""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]


def main():
    import workloads as W
    bpg = W._bpg()
    mode = sys.argv[1]
    if mode == "cache":
        bpg.lib().bpg_gens_cache_dir(sys.argv[2].encode())
        bpg.set_seed(5)
        syn = bpg.Synth(*W.config3())
        ctx = bpg.Context(0)
        proof, V = ctx.r1cs_prove(b"cache", syn.view, bytes(32))
        st = ctx.setup_stats()
        # the verifier never uses a set loaded from the file: it re-derives
        ok = ctx.r1cs_verify(b"cache", syn.view, V, proof)
        print(json.dumps({"proof": proof.hex(), **st, "verified": ok,
                          "from_cache_after_verify": ctx.setup_stats()["gens_from_cache"]}))
    else:
        # two circuit sizes proved at once from two threads on a fresh device
        # context: the larger one grows the generator set while the smaller
        # one's proofs are in flight (their snapshot must stay valid)
        stmts = {"small": W.config2(), "large": W.config3()}
        syns = {}
        for k, s in stmts.items():
            bpg.set_seed(9)
            syns[k] = bpg.Synth(*s)
        out = {k: [] for k in stmts}

        def run(k, reps):
            c = bpg.Context(0)
            for r in range(reps):
                out[k].append(c.r1cs_prove(b"conc", syns[k].view, bytes([r]) * 32)[0].hex())
        ts = [threading.Thread(target=run, args=("small", 6)), threading.Thread(target=run, args=("large", 2))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        print(json.dumps(out))


if __name__ == "__main__":
    main()
