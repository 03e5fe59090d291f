#!/bin/bash
# Kernel trace of the default bench (24 host threads) for the occupancy
# analysis (scripts/timeline.py over the middle of the run); the trace
# database stays in /tmp, only the summary comes back.
set -o pipefail
ROOTD=$(pwd)
R=${R:-r02m}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/${R}_trace
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/${R}_trace -o run -- python3 $ROOTD/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $ROOTD/gpurun_out/${R}_trace_bench.json 2> $ROOTD/gpurun_out/${R}_trace.err || exit $?
cd $ROOTD
python3 scripts/timeline.py /tmp/${R}_trace/run_results.db 0.35 gpurun_out/${R}_timeline.md 0.92 > /dev/null || exit $?
find /tmp/${R}_trace -name '*kernel_stats.csv' -exec cp {} gpurun_out/${R}_kernel_stats.csv \;
echo done
