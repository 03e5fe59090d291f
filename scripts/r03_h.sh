#!/bin/bash
# Round 3, call h: two proofs per consumer step with per-proof commitment
# jobs (less MSM scratch per workspace) through the batch tests, then A/B of
# consumer counts against one proof per step.
set -o pipefail
R=${R:-r03h}
mkdir -p gpurun_out
BPG_LOCKSTEP=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -x -v -k "batch" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
for rep in 1 2; do
  for v in "l1:BPG_LOCKSTEP=1:24" "l2c8:BPG_LOCKSTEP=2 BPG_PRODUCERS=8:16" "l2c12:BPG_LOCKSTEP=2 BPG_PRODUCERS=8:20" "l2c14:BPG_LOCKSTEP=2 BPG_PRODUCERS=8:22"; do
    name=${v%%:*}; rest=${v#*:}; envs=${rest%%:*}; thr=${rest#*:}
    env $envs timeout -k 10 600 python bench.py --steps 3 --warmup 1 --threads $thr --batch 384 --no-cpu-baseline > gpurun_out/${R}_ab_$name.json 2>> gpurun_out/${R}_ab.err || { echo "ab $name rc=$?" >> gpurun_out/${R}_ab.txt; continue; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$name.json'));print('$name', d['value'], d['ms_per_step'], d['host_cores_busy'], d['latency_ms_single_proof'], d.get('hbm_used_gb'))" >> gpurun_out/${R}_ab.txt
  done
done
echo done
