#!/bin/bash
# Round 3, call e: the lockstep prover (P = 1 for every path, then the batch
# tests with two proofs per consumer step), then A/B lockstep 1 vs 2.
set -o pipefail
R=${R:-r03e}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_gpu_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
BPG_LOCKSTEP=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_scale.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_lockstep2_tests.log 2>&1 || { echo "lockstep2 tests rc=$?"; exit 1; }
for rep in 1 2; do
  for v in 1 2; do
    BPG_LOCKSTEP=$v timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_l$v.json 2>> gpurun_out/${R}_ab.err || { echo "ab rc=$?"; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_l$v.json'));print('lockstep$v', d['value'], d['ms_per_step'], d['host_cores_busy'], d['latency_ms_single_proof'])" >> gpurun_out/${R}_ab.txt
  done
done
echo done
