#!/bin/bash
# Round 3, call q: wave priorities (s_setprio) for the latency-bound MSM tail
# kernels (pl2), plus the sort kernels (pls), plus the Straus triple fold
# (plsf), against the default build. MSM/fold parity of the most aggressive
# variant first, then ABCD x2 of the default bench command shortened to 3
# steps. Every GPU step has its own limit; the first failure ends the script.
set -o pipefail
R=${R:-r03q}
mkdir -p gpurun_out
V=$PWD/bulletproof-gadgets_amd/variants
BPG_LIB_PATH=$V/libbpg_plsf.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_parity_plsf.log 2>&1 || { echo "parity rc=$?"; exit 1; }
for rep in 1 2; do
  for v in base pl2 pls plsf; do
    unset BPG_LIB_PATH
    [ $v != base ] && export BPG_LIB_PATH=$V/libbpg_$v.so
    timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_$v.json 2>> gpurun_out/${R}_ab.err || { echo "ab $v rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$v.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['device_ms_by_kernel'])" >> gpurun_out/${R}_ab.txt
  done
done
echo done
