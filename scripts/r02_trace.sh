#!/bin/bash
# Kernel trace of the default bench (24 host threads) for the occupancy
# analysis (scripts/timeline.py over the middle of the run), without the
# bench's HIP-event bracketing (LIVE=1 turns it on: that combination crashed
# the profiler in hipEventRecord, profiles/r02p_prof_crash.txt); the trace
# database stays in /tmp, only the summary comes back.
set -o pipefail
ROOTD=$(pwd)
R=${R:-r02m}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/${R}_trace
BENCH_LIVE_TIMING=${LIVE:-0} timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/${R}_trace -o run -- python3 $ROOTD/bench.py --steps 3 --warmup 1 --no-cpu-baseline ${ARGS:-} > $ROOTD/gpurun_out/${R}_trace_bench.json 2> $ROOTD/gpurun_out/${R}_trace.err || exit $?
cd $ROOTD
db=$(find /tmp/${R}_trace -name '*.db' -print -quit)
python3 scripts/timeline.py "$db" 0.35 gpurun_out/${R}_timeline.md 0.92 > /dev/null || exit $?
python3 scripts/prof_summary.py "$db" gpurun_out/${R}_kernels.md > /dev/null || exit $?
# the same command without the profiler (bench live timing on) for comparison
timeout -k 10 600 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${ARGS:-} > gpurun_out/${R}_noprof_bench.json 2> gpurun_out/${R}_noprof.err || exit $?
echo done
