#!/bin/bash
# Round 3, call t: fourth priority A/B on top of the new default (tail 2,
# sort 3, misc 2, cached pass 1 at 1): the triple fold at 1 (f1), the comb
# fold at 1 (cb1), both with cached pass 1 at 2 (f1cb1c2); MSM pass 1 over the
# generators stays the only kernel at 0 in the last. Parity of f1cb1c2 first,
# then four variants x2 of the default bench command shortened to 3 steps.
# Every GPU step has its own limit; the first failure ends the script.
set -o pipefail
R=${R:-r03t}
mkdir -p gpurun_out
V=$PWD/bulletproof-gadgets_amd/variants
BPG_LIB_PATH=$V/libbpg_f1cb1c2.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_parity_f1cb1c2.log 2>&1 || { echo "parity rc=$?"; exit 1; }
for rep in 1 2; do
  for v in base f1 cb1 f1cb1c2; do
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
