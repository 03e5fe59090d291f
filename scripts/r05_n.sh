#!/bin/bash
# Round 5, call n: smoke + parity and statements tests, then A/B of the r05i
# build against the sort-scatter shuffle scans with the prepare gather on the
# null stream (no stream of its own).
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05n}
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_statements.py -m gpu -v --maxfail=3 \
    --timeout 300 --timeout-method thread > gpurun_out/${R}_tests.log 2>&1 &&
LIBS="c0989689:$V/libbpg_0989689.so head:" bash scripts/ab_lib.sh ${R} 3
