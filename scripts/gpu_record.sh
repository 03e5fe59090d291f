#!/bin/bash
# One round record in one gpurun call: smoke, the robustness module (process
# and thread exit) first, then the whole GPU suite, then the driver's bench
# command. Every step has its own time limit; the first failure ends the call.
# usage: scripts/gpu_record.sh <tag>   (outputs gpurun_out/<tag>_*)
set -o pipefail
mkdir -p gpurun_out
R=${1:?tag}
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_robustness.py -m gpu -v -x --timeout 240 --timeout-method thread \
    > gpurun_out/${R}_robust.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_gpu_tests.log 2>&1 &&
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
echo "rc=$?"
