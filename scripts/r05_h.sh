#!/bin/bash
# Round 5, call h: A/B of the build before the fused first-pass histogram
# (311e189) against it, then the batch verifier before its product tables
# and fused accumulation (2b7edd7) against it.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05h}
V=$PWD/bulletproof-gadgets_amd/variants
LIBS="c311e189:$V/libbpg_311e189.so head:" bash scripts/ab_lib.sh ${R} 3 &&
LIBS="c2b7edd:$V/libbpg_2b7edd7.so head:" bash scripts/ab_lib.sh ${R}_verify 2 --mode verify --steps 3 --warmup 1 --no-cpu-baseline
