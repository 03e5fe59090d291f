#!/bin/bash
# Round 3, call r: second priority A/B (sort kernels only at 1; tail at 2 with
# sort at 3; tail 2 + sort 1 again) and the final run sums taking over after
# two merge passes once <= 2^18 slots remain (BPG_RBK_STOP). MSM parity with
# BPG_RBK_STOP first (random, structured and one-bucket-heavy MSMs), then
# five variants x2 of the default bench command shortened to 3 steps, then
# the no-comb-table path once. Every GPU step has its own limit; the first
# failure ends the script.
set -o pipefail
R=${R:-r03r}
mkdir -p gpurun_out
V=$PWD/bulletproof-gadgets_amd/variants
BPG_RBK_STOP=262144 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_parity_stop.log 2>&1 || { echo "parity rc=$?"; exit 1; }
for rep in 1 2; do
  for v in base stop pls s1 pl2s3; do
    unset BPG_LIB_PATH BPG_RBK_STOP
    case $v in
      base) ;;
      stop) export BPG_RBK_STOP=262144 ;;
      *) export BPG_LIB_PATH=$V/libbpg_$v.so ;;
    esac
    timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_$v.json 2>> gpurun_out/${R}_ab.err || { echo "ab $v rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['device_ms_by_kernel'])" >> gpurun_out/${R}_ab.txt
  done
done
unset BPG_LIB_PATH BPG_RBK_STOP
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fold-tables 0 > gpurun_out/${R}_notables.json 2> gpurun_out/${R}_notables.err || { echo "notables rc=$?"; exit 1; }
echo done
