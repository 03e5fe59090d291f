#!/bin/bash
# One-GPU throughput under the per-rank CPU shares of an 8-rank node
# (VERDICT r03 item 1): the default, then the process pinned to 4 and 2 CPUs
# (an 8-rank run under a 32- and a 16-CPU quota).
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r04a
timeout -k 10 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline > $O.default.json 2> $O.default.err &&
timeout -k 10 300 taskset -c 0-3 python bench.py --steps 6 --warmup 1 --no-cpu-baseline > $O.cpus4.json 2> $O.cpus4.err &&
timeout -k 10 360 taskset -c 0-1 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O.cpus2.json 2> $O.cpus2.err
