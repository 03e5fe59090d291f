#!/bin/bash
# Round 3, call i: the lockstep-2 default (16 host threads: 8 RNG producers,
# 8 streams proving two proofs each) through smoke, the whole -m gpu suite,
# the driver's bench command, and that command under rocprofv3
# --kernel-trace --stats (kernel table + occupancy timeline). Every GPU step
# has its own limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r03i}
ROOTD=$(pwd)
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
(cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/${R}_prof && \
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/${R}_prof -o run -- python3 $ROOTD/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $ROOTD/gpurun_out/${R}_profdefault_bench.json 2> $ROOTD/gpurun_out/${R}_profdefault.err) || exit $?
db=$(find /tmp/${R}_prof -name '*.db' -print -quit)
python3 scripts/prof_summary.py "$db" gpurun_out/${R}_profdefault_kernels.md > /dev/null || exit $?
python3 scripts/timeline.py "$db" 0.35 gpurun_out/${R}_timeline_default.md 0.92 > /dev/null || exit $?
echo done
