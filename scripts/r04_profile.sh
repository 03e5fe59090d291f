#!/bin/bash
# Round 4 profiling call: smoke and the device parity module first (the
# build under profile must be bit-exact), then scripts/final_check.sh.
set -o pipefail
mkdir -p gpurun_out
R=${1:-r04m}
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${R}_parity.log 2>&1 &&
R=$R bash scripts/final_check.sh
