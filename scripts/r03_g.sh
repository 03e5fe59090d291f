#!/bin/bash
# Round 3, call g: zero-copy rows / c_L c_R (default) through the GPU tests,
# then A/B: zero copy on/off, two proofs per consumer step at 8 / 12 consumers.
set -o pipefail
R=${R:-r03g}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for rep in 1 2; do
  for v in "zc1:BPG_ZERO_COPY=1:24" "zc0:BPG_ZERO_COPY=0:24" "l2c8:BPG_LOCKSTEP=2 BPG_PRODUCERS=8:16" "l2c12:BPG_LOCKSTEP=2 BPG_PRODUCERS=8:20"; do
    name=${v%%:*}; rest=${v#*:}; envs=${rest%%:*}; thr=${rest#*:}
    env $envs timeout -k 10 600 python bench.py --steps 3 --warmup 1 --threads $thr --batch 384 --no-cpu-baseline > gpurun_out/${R}_ab_$name.json 2>> gpurun_out/${R}_ab.err || { echo "ab $name rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$name.json'));print('$name', d['value'], d['ms_per_step'], d['host_cores_busy'], d['latency_ms_single_proof'])" >> gpurun_out/${R}_ab.txt
  done
done
echo done
