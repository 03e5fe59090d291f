#!/bin/bash
# Round 4 experiments in one call: smoke + the GPU suite on the in-tree build
# (fixed-base MSM tables on by default, the lower-register row reduction),
# the single-proof latency, then the bench over three layouts in turn: the
# default, --msm-tables 0 (the ordinary 16-window jobs) and the triple fold
# with lazily loaded operands at 2 waves (variants/libbpg_lazy.so), twice.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04h}
VL=$PWD/bulletproof-gadgets_amd/variants/libbpg_lazy.so
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_gpu_tests.log 2>&1 &&
timeout -k 10 200 python bench.py --mode latency --steps 5 --warmup 1 > gpurun_out/${T}_latency.json 2> gpurun_out/${T}_latency.err || exit $?
for i in 1 2; do
  for v in default fb0 lazy; do
    L=; X=
    case $v in fb0) X="--msm-tables 0";; lazy) L=$VL;; esac
    BPG_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline $X > gpurun_out/${T}_ab_${v}_$i.json 2> gpurun_out/${T}_ab_${v}_$i.err || exit $?
  done
done
echo done
