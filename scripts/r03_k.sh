#!/bin/bash
# Round 3, call k: up to four proofs per consumer step (64-segment MSM jobs,
# binary segment search) through the batch / full-size tests at
# BPG_LOCKSTEP=4 and the default, then A/B x2: two proofs per step (default,
# 16 threads) against four per step with 4 / 6 consumers.
set -o pipefail
R=${R:-r03k}
mkdir -p gpurun_out
BPG_LOCKSTEP=4 timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_lockstep4_tests.log 2>&1 || { echo "lockstep4 tests rc=$?"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for rep in 1 2; do
  for v in "l2:BPG_LOCKSTEP=2:16" "l4c4:BPG_LOCKSTEP=4 BPG_PRODUCERS=8:12" "l4c6:BPG_LOCKSTEP=4 BPG_PRODUCERS=8:14"; do
    name=${v%%:*}; rest=${v#*:}; envs=${rest%%:*}; thr=${rest#*:}
    env $envs ${EXTRA_ENV:-} timeout -k 10 600 python bench.py --steps 3 --warmup 1 --threads $thr --batch 384 --no-cpu-baseline > gpurun_out/${R}_ab_$name.json 2>> gpurun_out/${R}_ab.err || { echo "ab $name rc=$?" >> gpurun_out/${R}_ab.txt; continue; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$name.json'));print('$name', d['value'], d['ms_per_step'], d['host_cores_busy'], d.get('hbm_used_gb'), d['roofline']['device_ms_by_kernel'])" >> gpurun_out/${R}_ab.txt
  done
done
echo done
