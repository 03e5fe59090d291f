#!/bin/bash
# Kernel trace of one throughput step for GPU occupancy analysis (busy union /
# concurrency, scripts/timeline.py). THREADS host threads (default 8: the
# profiler's tool library has crashed under 16 launching threads).
set -e
ROOTD=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/${R:-tr}_trace -o run -- python3 $ROOTD/bench.py --steps 1 --warmup 1 --no-cpu-baseline --threads ${THREADS:-8} > $ROOTD/gpurun_out/${R:-tr}_trace.json 2> $ROOTD/gpurun_out/${R:-tr}_trace.err
cd $ROOTD
python3 scripts/timeline.py gpurun_out/${R:-tr}_trace/run_results.db 0.3 gpurun_out/${R:-tr}_timeline.md > /dev/null
echo done
