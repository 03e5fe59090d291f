#!/bin/bash
# One-GPU lines (round 4): host RNG rates of the box's CPU, the single-proof
# latency, the driver's default command, the per-rank CPU shares of an
# 8-rank node (the process pinned to 4 and 2 CPUs: a 32- and a 16-CPU quota
# over 8 ranks), and the statements mode.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04d}
bulletproof-gadgets_amd/bin/rng_bench > gpurun_out/${T}_rng_bench.txt 2>&1 &&
timeout -k 10 200 python bench.py --mode latency --steps 5 --warmup 1 > gpurun_out/${T}_latency.json 2> gpurun_out/${T}_latency.err &&
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err &&
timeout -k 10 240 python bench.py --steps 5 --warmup 1 --cpus 4 --no-cpu-baseline > gpurun_out/${T}_cpus4.json 2> gpurun_out/${T}_cpus4.err &&
timeout -k 10 300 python bench.py --steps 4 --warmup 1 --cpus 2 --no-cpu-baseline > gpurun_out/${T}_cpus2.json 2> gpurun_out/${T}_cpus2.err &&
timeout -k 10 240 python bench.py --mode statements --steps 2 --warmup 1 > gpurun_out/${T}_statements.json 2> gpurun_out/${T}_statements.err
