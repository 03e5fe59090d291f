#!/usr/bin/env python3
"""CPU baseline at the bench's full size: the oracle (oracle/,
dalek's algorithms restated in C, one thread like the reference prover)
proving the config-5 statement (N = 2^20) on one host core, cold (generators
derived inside the call, as prove.rs:78 does on every prove) and warm.
Prints one JSON line; the bench's own cpu_baseline leg times a bounded
2^16 sample of the same family instead (minutes vs seconds).

usage: python scripts/cpu_baseline_full.py [config]
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]


def main():
    import threading
    t_start = time.perf_counter()

    def beat():   # a progress line a minute: the oracle call is silent for minutes
        while True:
            time.sleep(60)
            print("cpu_baseline_full: running, %.0f s" % (time.perf_counter() - t_start), file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    import oracle as O
    import workloads as W
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    bpg = W._bpg()
    inst, wit, gad = W.CONFIGS[cfg]()
    bpg.set_seed(1)
    syn = bpg.Synth(inst, wit, gad)
    L = O.lib()
    out = ctypes.create_string_buffer(417 + 64 * 31)
    plen = ctypes.c_size_t(0)
    V = ctypes.create_string_buffer(32 * max(syn.m, 1))
    view = ctypes.cast(ctypes.addressof(syn.view), ctypes.POINTER(O.R1csView))
    t0 = time.perf_counter()
    L.oracle_r1cs_prove(b"bench", 5, view, b"\1" * 32, out, len(out), ctypes.byref(plen), V)
    cold = time.perf_counter() - t0
    t0 = time.perf_counter()
    L.oracle_r1cs_prove(b"bench", 5, view, b"\2" * 32, out, len(out), ctypes.byref(plen), V)
    warm = time.perf_counter() - t0
    model = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), "?")
    print(json.dumps({"config": cfg, "n": syn.n, "q": syn.q, "cores": 1, "kind": "port",
                      "cold_s": round(cold, 1), "warm_s": round(warm, 1),
                      "constraints_per_s_cold": round(syn.q / cold, 1), "constraints_per_s_warm": round(syn.q / warm, 1),
                      "cpu_model": model, "nproc": os.cpu_count()}), flush=True)


if __name__ == "__main__":
    main()
