#!/bin/bash
# Round 4: fixed-base generator tables (variants/libbpg_fb.so): parity tests
# on that library, then the bench A/B/A/B against the in-tree default.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04f}
V=$PWD/bulletproof-gadgets_amd/variants/libbpg_fb.so
BPG_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_scale.py \
    -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/${T}_fb_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_ab_default_$i.json 2> gpurun_out/${T}_ab_default_$i.err || exit $?
  BPG_LIB_PATH=$V timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_ab_fb_$i.json 2> gpurun_out/${T}_ab_fb_$i.err || exit $?
done
echo done
