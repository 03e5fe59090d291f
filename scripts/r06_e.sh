#!/bin/bash
# Round 6, call e: smoke + whole GPU suite on the comb-fold arguments by value,
# the fused small-row reduction and the one-launch triple fold; the default
# command under rocprofv3 (launches per proof); A/B of the round-5 build.
set -o pipefail
mkdir -p gpurun_out
R=r06e
V=$PWD/bulletproof-gadgets_amd/variants
ROOTD=$(pwd)
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/${R}_prof && \
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/${R}_prof -o run -- python3 $ROOTD/bench.py --steps 3 --warmup 1 --no-cpu-baseline --isolated-proofs 0 > $ROOTD/gpurun_out/${R}_profdefault_bench.json 2> $ROOTD/gpurun_out/${R}_profdefault.err) &&
python3 scripts/prof_summary.py $(find /tmp/${R}_prof -name '*.db' -print -quit) gpurun_out/${R}_profdefault_kernels.md > /dev/null &&
LIBS="r05:$V/libbpg_r05.so head:" bash scripts/ab_lib.sh ${R} 2 --steps 5 --warmup 2 --no-cpu-baseline --isolated-proofs 0
echo "rc=$?"
