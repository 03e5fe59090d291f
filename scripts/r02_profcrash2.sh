#!/bin/bash
# rocprofv3 --kernel-trace crash bisection with round triples on:
# A: IPP tail from level 2 on (no depth-2 MSM jobs, no fold3);
# B: default schedule without the bench's HIP-event bracketing.
ROOTD=$(pwd)
R=${R:-r02o}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pcA
BPG_IPP_TAIL=300000 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pcA -o run -- python3 $ROOTD/bench.py --steps 1 --warmup 1 --batch 32 --no-cpu-baseline > $ROOTD/gpurun_out/${R}_A.json 2> $ROOTD/gpurun_out/${R}_A.err
echo "A rc=$?" >> $ROOTD/gpurun_out/${R}_rc.txt
rm -rf /tmp/pcB
BENCH_LIVE_TIMING=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pcB -o run -- python3 $ROOTD/bench.py --steps 1 --warmup 1 --batch 32 --no-cpu-baseline > $ROOTD/gpurun_out/${R}_B.json 2> $ROOTD/gpurun_out/${R}_B.err
echo "B rc=$?" >> $ROOTD/gpurun_out/${R}_rc.txt
echo done
