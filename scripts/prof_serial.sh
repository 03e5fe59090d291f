#!/bin/bash
# Kernel durations without stream overlap: bench with one consumer stream
# (2 host threads) under rocprofv3 --kernel-trace --stats.
set -e
ROOTD=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/${R:-ser}_prof -o run -- python3 $ROOTD/bench.py --steps 1 --warmup 1 --no-cpu-baseline --threads 2 --batch ${BATCH:-4} > $ROOTD/gpurun_out/${R:-ser}_prof.json 2> $ROOTD/gpurun_out/${R:-ser}_prof.err
cd $ROOTD
python3 scripts/prof_summary.py gpurun_out/${R:-ser}_prof/run_results.db gpurun_out/${R:-ser}_prof_kernels.md > /dev/null
echo done
