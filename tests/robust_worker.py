"""Child process of tests/test_gpu_robustness.py (a fresh device context per
run). usage: robust_worker.py cache <dir> | concurrent | exit | queues |
stmts_hbm <GB> | stmts_oom"""
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
        # no wait here: the process exits while the OS threads may still be
        # running their thread-exit code (the round-4 SIGSEGV's window)
        print(json.dumps(dict(out, park=bpg.Context(0).setup_stats())), flush=True)


def exit_with_live_workspaces():
    """The low-HBM path (no comb tables) on three threads, and an exit with
    device workspaces still owned: the main thread's (its thread_local
    destructors run inside exit()), one finished thread's, and one thread
    still alive (blocked) when the process exits."""
    import workloads as W
    bpg = W._bpg()
    bpg.set_seed(3)
    syn = bpg.Synth(*W.config3())
    ctx = bpg.Context(0)
    ctx.set_strategy(fold_tables=0)
    hold = threading.Event()
    out = {}

    def prove(k, block):
        out[k] = ctx.r1cs_prove(b"exit", syn.view, bytes([len(k)]) * 32)[0].hex()
        if block:
            hold.wait()   # never set: alive at exit
    done = threading.Thread(target=prove, args=("done", False))
    live = threading.Thread(target=prove, args=("live", True), daemon=True)
    done.start()
    live.start()
    prove("main", False)
    done.join()
    while "live" not in out:
        hold.wait(0.05)
    print(json.dumps(dict(out, park=ctx.setup_stats())), flush=True)


def queues():
    """A batch under HIP's default hardware queues (the parent removes
    GPU_MAX_HW_QUEUES): the library sizes its consumer streams to the queues
    it has, and the proofs equal single proofs."""
    import workloads as W
    bpg = W._bpg()
    bpg.set_seed(6)
    syn = bpg.Synth(*W.config2())
    ctx = bpg.Context(0)
    prep = ctx.prepare(syn.view)
    ents = [bytes([k + 90]) * 32 for k in range(40)]
    proofs = prep.prove_batch(b"queues", ents, threads=14)
    st = bpg.last_batch_stats()
    same = all(proofs[k] == ctx.r1cs_prove(b"queues", syn.view, ents[k])[0] for k in (0, 17, 39))
    print(json.dumps({"stats": st, "same": same, "distinct": len(set(proofs))}), flush=True)


def stmts_hbm(foreign_gb):
    """bpg_prove_statements at 12 device threads of four (16 hardware
    queues) next to a foreign allocation of `foreign_gb` GB in this process:
    the call must complete, or fail with an error, never abort its queues."""
    import torch
    import workloads as W
    bpg = W._bpg()
    free, _ = torch.cuda.mem_get_info(0)
    hog = torch.empty(hog_bytes(foreign_gb, free), dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    free_after, _ = torch.cuda.mem_get_info(0)
    texts = [W.config5(70000 + i) for i in range(24)]
    bpg.set_statements_layout(12, 4)
    err = None
    try:
        outs = bpg.prove_statements("hbm", texts, 16)
    except bpg.BpgError as e:
        outs, err = [], str(e)
    st = bpg.last_statements_stats()
    ok = [o is not None for o in outs]
    ver = bool(outs) and outs[-1] is not None and bpg.verify("hbm", texts[-1][0], outs[-1][0], outs[-1][1], texts[-1][2])
    del hog
    print(json.dumps({"proved": sum(ok), "count": len(texts), "error": err, "last_error": bpg.last_error(),
                      "stats": st, "verified_last": ver, "foreign_gb": round(hog_bytes(foreign_gb, free) / 1e9, 1),
                      "free_gb_before": round(free / 1e9, 1), "free_gb_after_foreign": round(free_after / 1e9, 1)}),
          flush=True)


def stmts_oom():
    """bpg_prove_statements with three device threads while the parent's
    BPG_TEST_INJECT_OOM makes the first proof to reach that IPP round throw
    hipErrorOutOfMemory half way through gpu_prove_lockstep: that device
    thread hands its statements back, frees its workspace and retires
    (ADVICE r5), the others prove them, and every proof must still equal
    the statement's own sequential c_prove."""
    import workloads as W
    bpg = W._bpg()
    sts = [W.config2(4100 + k) for k in range(12)]
    seeds = [500 + k for k in range(len(sts))]
    bpg.set_statements_layout(3, 2)
    err = None
    try:
        outs = bpg.prove_statements("oom", sts, 6, seeds=seeds)
    except bpg.BpgError as e:
        outs, err = [], str(e)
    st = bpg.last_statements_stats()
    same = []
    for k, (s, seed) in enumerate(zip(sts, seeds)):
        if k < len(outs):
            bpg.set_seed(seed)
            same.append(outs[k] is not None and outs[k] == bpg.prove("oom", *s))
    print(json.dumps({"proved": sum(o is not None for o in outs), "count": len(sts), "error": err,
                      "stats": st, "same": same}), flush=True)


def hog_bytes(gb, free):
    return int(min(gb * 1e9, free - 40e9))


if __name__ == "__main__":
    if sys.argv[1] == "stmts_hbm":
        stmts_hbm(float(sys.argv[2]))
        sys.exit(0)
    if sys.argv[1] == "stmts_oom":
        stmts_oom()
        sys.exit(0)
    if sys.argv[1] == "queues":
        queues()
        sys.exit(0)
    if sys.argv[1] == "exit":
        sys.path[:0] = [ROOT]
        exit_with_live_workspaces()
        sys.exit(0)
    main()
