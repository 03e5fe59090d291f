#!/bin/bash
# Parity of the default build (comb radix 2^COMB_BITS) on the fold tests and
# the full-size goldens, then A/B bench lines: default vs the variants listed
# in AB (name=libpath), alternating.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02e}
# PARITY_LIB: run the parity tests on that variant library instead of the default
# SKIP_PARITY=1: the caller ran the tests already
if [ "${SKIP_PARITY:-0}" != 1 ]; then
if [ -n "$PARITY_LIB" ]; then export BPG_LIB_PATH=$PARITY_LIB; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py "tests/test_gpu_parity.py::test_fold_strategy_bit_exact" \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${R}_parity.log 2>&1 || exit $?
unset BPG_LIB_PATH
fi
for rep in 1 2; do
  for v in default $AB; do
    name=${v%%=*}; lib=${v#*=}
    if [ "$name" = default ]; then unset BPG_LIB_PATH; else export BPG_LIB_PATH=$lib; fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_${name}_$rep.json 2> gpurun_out/${R}_ab_${name}_$rep.err || exit $?
    echo "$name $rep $(python3 -c "import json; d=json.loads(open('gpurun_out/${R}_ab_${name}_$rep.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['cold_setup_ms'], d['roofline']['device_ms_by_kernel'].get('ipp_comb_fold'))")" >> gpurun_out/${R}_ab_summary.txt
  done
done
unset BPG_LIB_PATH
echo done
