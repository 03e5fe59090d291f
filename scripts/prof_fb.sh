#!/bin/bash
# Kernel trace of the fold/MSM microbenchmark.
set -e
ROOTD=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $ROOTD/gpurun_out/${R:-fb}_prof -o run -- $ROOTD/bulletproof-gadgets_amd/bin/fold_bench_w2 > $ROOTD/gpurun_out/${R:-fb}_prof.log 2>&1
echo done
