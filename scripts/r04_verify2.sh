#!/bin/bash
# Verification with chunks of clamp(ceil(count / 6), 8, 64): the device
# verifier tests, then the verify bench at its default batch.
set -o pipefail
mkdir -p gpurun_out
R=${1:-r04z}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_matrix.py tests/test_gpu_scale.py \
    -m gpu -v -x --timeout 300 --timeout-method thread -k "verify or matrix" > gpurun_out/${R}_verify_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/${R}_verify.json 2> gpurun_out/${R}_verify.err
echo "rc=$?"
