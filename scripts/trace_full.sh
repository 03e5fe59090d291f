#!/bin/bash
# Kernel trace of one throughput step (16 host threads, batch 128) for GPU
# occupancy analysis (busy union / concurrency).
set -e
ROOTD=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace -d $ROOTD/gpurun_out/${R:-tr}_trace -o run -- python3 $ROOTD/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $ROOTD/gpurun_out/${R:-tr}_trace.json 2> $ROOTD/gpurun_out/${R:-tr}_trace.err
echo done
