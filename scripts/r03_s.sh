#!/bin/bash
# Round 3, call s: third priority A/B on top of the new default (tail 2,
# sort 3): the scalar-vector kernels between MSM jobs at 2 (m2), those and
# the tail at 3 (m3l3), m2 with MSM pass 1 over cached bases at 1 (m2c1).
# Parity of m3l3 first, then four variants x2 of the default bench command
# shortened to 3 steps. Every GPU step has its own limit; the first failure
# ends the script.
set -o pipefail
R=${R:-r03s}
mkdir -p gpurun_out
V=$PWD/bulletproof-gadgets_amd/variants
BPG_LIB_PATH=$V/libbpg_m3l3.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_parity_m3l3.log 2>&1 || { echo "parity rc=$?"; exit 1; }
for rep in 1 2; do
  for v in base m2 m3l3 m2c1; do
    unset BPG_LIB_PATH
    case $v in
      base) ;;
      *) export BPG_LIB_PATH=$V/libbpg_$v.so ;;
    esac
    timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_$v.json 2>> gpurun_out/${R}_ab.err || { echo "ab $v rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['device_ms_by_kernel'])" >> gpurun_out/${R}_ab.txt
  done
done
unset BPG_LIB_PATH
echo done
