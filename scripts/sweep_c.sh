#!/bin/bash
# Throughput vs consumer streams (producers fixed at 8).
set -e
mkdir -p gpurun_out
for T in 9 10 12 16; do
  BPG_PRODUCERS=8 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --threads $T --batch 64 --no-cpu-baseline > gpurun_out/swc_t$T.json 2> gpurun_out/swc_t$T.err
done
echo done
