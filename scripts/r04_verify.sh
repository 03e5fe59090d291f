#!/bin/bash
# Batched verification (one random-linear-combination MSM per chunk): the
# device verifier tests, then the verify bench and the single-verification
# bench.
set -o pipefail
mkdir -p gpurun_out
R=${1:-r04r}
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_matrix.py tests/test_gpu_scale.py \
    -m gpu -v -x --timeout 300 --timeout-method thread -k "verify or matrix or reject or fixture" \
    > gpurun_out/${R}_verify_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/${R}_verify.json 2> gpurun_out/${R}_verify.err &&
timeout -k 10 300 python bench.py --mode verify-sharded --steps 20 --warmup 3 > gpurun_out/${R}_verify_sharded.json 2> gpurun_out/${R}_verify_sharded.err
echo "rc=$?"
