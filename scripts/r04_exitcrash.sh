#!/bin/bash
# The concurrent-sizes worker (tests/robust_worker.py) under Python's
# faulthandler: with the per-proof scalar launches (in-tree build), then with
# the round's a/b folds and tail weights batched over the lockstep proofs
# (variants/libbpg_batched.so), then the robustness tests on the in-tree build.
set -o pipefail
mkdir -p gpurun_out
R=${1:-r04w}
timeout -k 10 250 python -X faulthandler tests/robust_worker.py concurrent > gpurun_out/${R}_main.out 2> gpurun_out/${R}_main.err
echo "rc=$?" >> gpurun_out/${R}_main.err
BPG_LIB_PATH=$PWD/bulletproof-gadgets_amd/variants/libbpg_batched.so timeout -k 10 250 python -X faulthandler tests/robust_worker.py concurrent > gpurun_out/${R}_batched.out 2> gpurun_out/${R}_batched.err
echo "rc=$?" >> gpurun_out/${R}_batched.err
timeout -k 10 400 python -u -m pytest tests/test_gpu_robustness.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${R}_robust.log 2>&1
echo "rc=$?"
