#!/bin/bash
# GPU test suite + smoke + the single-proof latency line on one box (round 4).
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04b}
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 400 --timeout-method thread \
    > gpurun_out/${T}_gpu_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --mode latency --steps 5 --warmup 1 > gpurun_out/${T}_latency.json 2> gpurun_out/${T}_latency.err
