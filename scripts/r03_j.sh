#!/bin/bash
# Round 3, call j: folds with T-less additions (before doublings) and the
# bucket-segment length switch through the parity tests, then ABCD x2:
# A the previous build (variant lib), B the new build, C / D with 16 / 32
# buckets per first-level segment (BPG_MSM_SEGLEN).
set -o pipefail
R=${R:-r03j}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
BPG_MSM_SEGLEN=32 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "msm or batch or full_size" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_seg32_tests.log 2>&1 || { echo "seg32 tests rc=$?"; exit 1; }
V=$PWD/bulletproof-gadgets_amd/variants
for rep in 1 2; do
  for v in A B C D; do
    unset BPG_LIB_PATH BPG_MSM_SEGLEN
    case $v in
      A) export BPG_LIB_PATH=$V/libbpg_base.so ;;
      C) export BPG_MSM_SEGLEN=16 ;;
      D) export BPG_MSM_SEGLEN=32 ;;
    esac
    timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_$v.json 2>> gpurun_out/${R}_ab.err || { echo "ab $v rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['device_ms_by_kernel'])" >> gpurun_out/${R}_ab.txt
  done
done
echo done
