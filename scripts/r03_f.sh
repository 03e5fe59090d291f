#!/bin/bash
# Round 3, call f: the batch tests with two proofs per consumer step, then
# A/B: lockstep 1 / 2, with device RNG slots or pinned host slots.
set -o pipefail
R=${R:-r03f}
mkdir -p gpurun_out
BPG_LOCKSTEP=2 timeout -k 10 700 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_lockstep2_tests.log 2>&1 || { echo "lockstep2 tests rc=$?"; exit 1; }
BPG_LOCKSTEP=2 BPG_HOST_SLOTS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -v -k batch --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_hostslots_tests.log 2>&1 || { echo "hostslots tests rc=$?"; exit 1; }
for rep in 1 2; do
  for v in "l1:BPG_LOCKSTEP=1" "l2:BPG_LOCKSTEP=2" "l2h:BPG_LOCKSTEP=2 BPG_HOST_SLOTS=1" "l1h:BPG_LOCKSTEP=1 BPG_HOST_SLOTS=1"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_$name.json 2>> gpurun_out/${R}_ab.err || { echo "ab $name rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$name.json'));print('$name', d['value'], d['ms_per_step'], d['host_cores_busy'], d['latency_ms_single_proof'])" >> gpurun_out/${R}_ab.txt
  done
done
echo done
