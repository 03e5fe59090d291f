#!/bin/bash
# Round-2 bench pass: the driver's own command (steps 20, warmup 5), then the
# default-thread-count bench under rocprofv3 kernel tracing (round 1 saw a
# profiler SIGSEGV at 16 host threads; BENCH_LIVE_TIMING=0 first isolates the
# bench's own HIP-event bracketing from the profiler).
set -o pipefail
R=${R:-r02a}
mkdir -p gpurun_out
ROOTD=$(pwd)
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
cd /tmp && export TMPDIR=/tmp
BENCH_LIVE_TIMING=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/${R}_prof_nolive -o run -- \
  python3 $ROOTD/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOTD/gpurun_out/${R}_prof_nolive.json 2> $ROOTD/gpurun_out/${R}_prof_nolive.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/${R}_prof -o run -- \
  python3 $ROOTD/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOTD/gpurun_out/${R}_prof.json 2> $ROOTD/gpurun_out/${R}_prof.err || exit $?
echo done
