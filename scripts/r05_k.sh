#!/bin/bash
# Round 5, call k: smoke + GPU suite, then A/B of the committed build
# (0989689) against the 1024-thread fused digit launch, the prefetching
# column scan and the device-side equal-scalar gather at prepare: the
# driver's bench, then statements mode.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05k}
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_gpu_tests.log 2>&1 &&
LIBS="c0989689:$V/libbpg_0989689.so head:" bash scripts/ab_lib.sh ${R} 2 &&
LIBS="c0989689:$V/libbpg_0989689.so head:" bash scripts/ab_lib.sh ${R}_stmts 2 --mode statements --steps 2 --warmup 1 --no-cpu-baseline
