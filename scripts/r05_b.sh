#!/bin/bash
# Round 5, call b: the whole GPU suite on the current build, then A/B of the
# round-4 library against it (ABAB).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05b_smoke.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/r05b_gpu_tests.log 2>&1 &&
LIBS="r04:$PWD/bulletproof-gadgets_amd/variants/libbpg_r04.so head:" bash scripts/ab_lib.sh r05b 2
