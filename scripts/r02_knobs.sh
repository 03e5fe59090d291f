#!/bin/bash
# Parity of the current build (fold strategies on small fixtures, full-size
# goldens), then bench lines for run-time knobs: default, 20 host threads,
# IPP tail threshold 2048 / 8192, the all-stable radix sort variant.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02k}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${R}_parity.log 2>&1 || exit $?
run() {   # name, env assignments..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline $EXTRA > gpurun_out/${R}_${name}.json 2> gpurun_out/${R}_${name}.err || return $?
  echo "$name $(python3 -c "import json; d=json.loads(open('gpurun_out/${R}_${name}.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['latency_ms_single_proof'], d['cold_setup_ms'], d['host_cores_busy'])")" >> gpurun_out/${R}_summary.txt
}
run default BPG_X=0 || exit $?
EXTRA="--threads 20" run threads20 BPG_X=0 || exit $?
run tail2048 BPG_IPP_TAIL=2048 || exit $?
run stablesort BPG_LIB_PATH=bulletproof-gadgets_amd/variants/libbpg_ss.so || exit $?
run tail8192 BPG_IPP_TAIL=8192 || exit $?
run default2 BPG_X=0 || exit $?
echo done
