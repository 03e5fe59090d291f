#!/bin/bash
# Round 4 experiments in one call: smoke, the MSM/fixture parity subset, one
# bench per layout (the default with fixed-base MSM tables from 2^18
# generators, --msm-tables 0, and the triple fold with lazily loaded operands
# at 2 waves from variants/libbpg_lazy.so), the single-proof latency, then
# the whole GPU suite.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04h}
VL=$PWD/bulletproof-gadgets_amd/variants/libbpg_lazy.so
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -x --timeout 120 --timeout-method thread \
    -k "msm or fixture_bit_exact" > gpurun_out/${T}_parity.log 2>&1 || exit $?
for v in default fb0 lazy; do
  L=; X=
  case $v in fb0) X="--msm-tables 0";; lazy) L=$VL;; esac
  BPG_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $X > gpurun_out/${T}_ab_${v}.json 2> gpurun_out/${T}_ab_${v}.err || exit $?
done
timeout -k 10 200 python bench.py --mode latency --steps 5 --warmup 1 > gpurun_out/${T}_latency.json 2> gpurun_out/${T}_latency.err &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_gpu_tests.log 2>&1
echo "rc=$?"
