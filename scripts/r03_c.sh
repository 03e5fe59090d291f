#!/bin/bash
# Round 3, call c: GPU tests on the single commitment job, then an ABCD x2
# A/B: default (one commitment job) / two jobs / fold3 at 2 waves without
# and with the entry prefetch (variant builds, two commitment jobs).
set -o pipefail
R=${R:-r03c}
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_gpu_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
fi
BPG_SMALL_MSM=20000 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_statements.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_smsm_tests.log 2>&1 || { echo "smsm tests rc=$?"; exit 1; }
V=$PWD/bulletproof-gadgets_amd/variants
for rep in 1 2; do
  for v in A B C D E; do
    unset BPG_LIB_PATH BPG_COMMIT_ONE_JOB BPG_SMALL_MSM
    case $v in
      B) export BPG_COMMIT_ONE_JOB=0 ;;
      C) export BPG_LIB_PATH=$V/libbpg_f3w2p0.so ;;
      D) export BPG_LIB_PATH=$V/libbpg_f3w2p1.so ;;
      E) export BPG_SMALL_MSM=20000 ;;
    esac
    timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_$v.json 2>> gpurun_out/${R}_ab.err || { echo "ab rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['device_ms_by_kernel'])" >> gpurun_out/${R}_ab.txt
  done
done
echo done
