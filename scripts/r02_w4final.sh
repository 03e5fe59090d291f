#!/bin/bash
# A/B of MSM pass 1 compiled for 4 waves per SIMD (RBK_WAVES=4: 128 VGPRs,
# 88 B/lane scratch) against the default 3, ABAB on one box; then the
# round-end profiles of the current build: 8-thread kernel trace + occupancy
# timeline, and the PMC passes. Every GPU step has its own time limit; the
# first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02zz}
rm -f gpurun_out/ab_summary.txt
STEPS=3 VARIANTS="d1:X=1 w4a:BPG_LIB_PATH=bulletproof-gadgets_amd/variants/libbpg_w4.so d2:X=1 w4b:BPG_LIB_PATH=bulletproof-gadgets_amd/variants/libbpg_w4.so" bash scripts/ab.sh || exit $?
R=${R}_t8 ARGS='--threads 8' bash scripts/r02_trace.sh || exit $?
R=${R} ARGS="--steps 1 --warmup 1 --threads 8 --batch 32 --no-cpu-baseline" bash scripts/r02_pmc.sh || exit $?
echo done
