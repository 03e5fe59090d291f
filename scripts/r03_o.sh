#!/bin/bash
# Round 3, call o: the row reduction with three points live (sum of A_s added
# after the scan; 225 instead of 266 VGPRs) through the MSM / full-size
# parity tests, then ABC x2: A the previous build, B the new one, C the new
# one with the MSM window width from the multiply-count model (with four
# proofs per job the IPP jobs hold 8 MSMs), then the statements mode.
set -o pipefail
R=${R:-r03o}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
BPG_MSM_WINDOW_MODEL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -k "msm or batch or full_size" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_model_tests.log 2>&1 || { echo "model tests rc=$?"; exit 1; }
V=$PWD/bulletproof-gadgets_amd/variants
for rep in 1 2; do
  for v in A B C; do
    unset BPG_LIB_PATH BPG_MSM_WINDOW_MODEL
    case $v in
      A) export BPG_LIB_PATH=$V/libbpg_base.so ;;
      C) export BPG_MSM_WINDOW_MODEL=1 ;;
    esac
    timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_$v.json 2>> gpurun_out/${R}_ab.err || { echo "ab $v rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['device_ms_by_kernel'])" >> gpurun_out/${R}_ab.txt
  done
done
unset BPG_LIB_PATH BPG_MSM_WINDOW_MODEL
timeout -k 10 600 python bench.py --mode statements --steps 2 --warmup 1 > gpurun_out/${R}_statements.json 2> gpurun_out/${R}_statements.err || exit $?
echo done
