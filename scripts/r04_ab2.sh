#!/bin/bash
# A/B: MSM pass 1 over cached bases compiled for 3 waves per SIMD (168
# VGPRs, 8 spilled; variants/libbpg_cw3.so) against the default 2 (176),
# alternated twice; then the default at 4 and 2 CPUs (per-rank shares of an
# 8-rank node under 32- and 16-CPU quotas), then statements at 8, 12, 16 device threads.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04n}
V=$PWD/bulletproof-gadgets_amd/variants/libbpg_cw3.so
for i in 1 2; do
  for v in default cw3; do
    L=; [ $v = cw3 ] && L=$V
    BPG_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_ab_${v}_$i.json 2> gpurun_out/${T}_ab_${v}_$i.err || exit $?
  done
done
for c in 4 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --cpus $c > gpurun_out/${T}_cpus$c.json 2> gpurun_out/${T}_cpus$c.err || exit $?
done
echo done
for c in 8 12 16; do
  timeout -k 10 400 python bench.py --mode statements --steps 2 --warmup 1 --consumers $c > gpurun_out/${T}_stmts_c$c.json 2> gpurun_out/${T}_stmts_c$c.err || exit $?
done
echo done2
