#!/bin/bash
# Round 5, call c: smoke + whole GPU suite on the current build, A/B of the
# previous tested build (r05b) against it, then a rocprofv3 kernel trace of
# the default bench command (launches per proof, kernel shares).
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05c}
ROOTD=$(pwd)
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_gpu_tests.log 2>&1 &&
LIBS="r05b:$PWD/bulletproof-gadgets_amd/variants/libbpg_r05b.so head:" bash scripts/ab_lib.sh ${R} 2 || exit $?
(cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/${R}_prof && \
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/${R}_prof -o run -- python3 $ROOTD/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $ROOTD/gpurun_out/${R}_profdefault_bench.json 2> $ROOTD/gpurun_out/${R}_profdefault.err) || exit $?
db=$(find /tmp/${R}_prof -name '*.db' -print -quit)
python3 scripts/prof_summary.py "$db" gpurun_out/${R}_profdefault_kernels.md > /dev/null || exit $?
python3 scripts/timeline.py "$db" 0.35 gpurun_out/${R}_timeline_default.md 0.92 > /dev/null || exit $?
timeout -k 10 180 bulletproof-gadgets_amd/bin/affine_bench > gpurun_out/${R}_affine_bench.txt 2>&1 || exit $?
echo done
