#!/bin/bash
# Round-3 GPU check: parity tests (incl. the sharded full-size golden cases),
# smoke, a short default bench, the prepared sharded verifier at 1 rank, and
# the producer-stream A/B. Every GPU step has its own limit; the first failure
# ends the script.
set -o pipefail
R=${R:-r03a}
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider ${TEST_ARGS:-} > gpurun_out/${R}_gpu_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
fi
if [ "${SMOKE:-1}" = 1 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { echo "smoke rc=$?"; exit 1; }
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py --gpus 1 --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS:-} > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || { echo "bench rc=$?"; exit 1; }
fi
if [ "${VSH:-1}" = 1 ]; then
  timeout -k 10 300 python bench.py --mode verify-sharded --steps 20 --warmup 3 > gpurun_out/${R}_verify_sharded.json 2> gpurun_out/${R}_verify_sharded.err || { echo "vsh rc=$?"; exit 1; }
fi
if [ "${AB:-0}" = 1 ]; then
  for v in 0 1 0 1; do
    BPG_PRODUCER_STREAMS=$v timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_ps$v.json 2>> gpurun_out/${R}_ab.err || { echo "ab rc=$?"; exit 1; }
    python3 -c "import json,sys;d=json.load(open('gpurun_out/${R}_ab_ps$v.json'));print('$v', d['value'], d['ms_per_step'])" >> gpurun_out/${R}_ab.txt
  done
fi
echo done
