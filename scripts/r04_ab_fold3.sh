#!/bin/bash
# Round 4: the triple fold with its table operands loaded lazily (2 waves per
# SIMD, variants/libbpg_lazy.so) against the default (1 wave, 332 registers):
# isolated timing + correctness, then the bench A/B/A/B; plus the host RNG
# rates and the single-proof latency of the default build.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04e}
B=bulletproof-gadgets_amd/bin
$B/rng_bench > gpurun_out/${T}_rng_bench.txt 2>&1 &&
timeout -k 10 120 $B/fold3_bench > gpurun_out/${T}_fold3_default.txt 2>&1 &&
timeout -k 10 120 $B/fold3_bench_lazy > gpurun_out/${T}_fold3_lazy.txt 2>&1 &&
timeout -k 10 200 python bench.py --mode latency --steps 5 --warmup 1 > gpurun_out/${T}_latency.json 2> gpurun_out/${T}_latency.err || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_ab_default_$i.json 2> gpurun_out/${T}_ab_default_$i.err || exit $?
  BPG_LIB_PATH=$PWD/bulletproof-gadgets_amd/variants/libbpg_lazy.so timeout -k 10 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_ab_lazy_$i.json 2> gpurun_out/${T}_ab_lazy_$i.err || exit $?
done
echo done
