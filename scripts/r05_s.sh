#!/bin/bash
# Round 5, call s: the column scan's per-256 form (all 2,048 loads issued
# first, one barrier per 256) on the final build, against the final build.
# Its earlier A/Bs (r05k, r05l) also carried a prepare-time stream that cost
# -1.3% on its own (r05m), so they did not isolate it.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05s}
V=$PWD/bulletproof-gadgets_amd/variants
LIBS="head: scan2:$V/libbpg_scan2.so" bash scripts/ab_lib.sh ${R} 3
