#!/bin/bash
# Round 3, call d: GPU tests on the window cost model + in-kernel tile table,
# then A/B: window model on/off, and host threads / hardware queues.
set -o pipefail
R=${R:-r03d}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_gpu_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
run() {   # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $BARGS > gpurun_out/${R}_ab_$name.json 2>> gpurun_out/${R}_ab.err || { echo "ab $name rc=$?"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$name.json'));print('$name', d['value'], d['ms_per_step'], d['config']['host_threads_per_gpu'], d['host_cores_busy'])" >> gpurun_out/${R}_ab.txt
}
for rep in 1 2; do
  BARGS="" run model1 BPG_MSM_WINDOW_MODEL=1
  BARGS="" run model0 BPG_MSM_WINDOW_MODEL=0
done
BARGS="--threads 28" run t28q16 GPU_MAX_HW_QUEUES=16
BARGS="--threads 28" run t28q20 GPU_MAX_HW_QUEUES=20
BARGS="" run t24q16 GPU_MAX_HW_QUEUES=16
BARGS="--threads 32" run t32q24 GPU_MAX_HW_QUEUES=24
echo done
