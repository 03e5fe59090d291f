#!/bin/bash
# Throughput sweep on the GPU box: RNG rate per thread, then bench at several
# host-thread / producer splits. Output under gpurun_out/sweep_*.
set -e
mkdir -p gpurun_out
echo "cpus: $(nproc) affinity: $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')" > gpurun_out/sweep_env.txt
lscpu | grep -E "Model name|Socket|Core|Thread" >> gpurun_out/sweep_env.txt || true
timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.')
import workloads as W
L = W._bpg().lib()
import ctypes
L.bpg_rng_rate.restype = ctypes.c_double
for lanes in (1, 8):
    print('rng draws/s/thread lanes=%d: %.3g' % (lanes, L.bpg_rng_rate(200000, lanes)))
" >> gpurun_out/sweep_env.txt
for cfg in ${CFGS:-"16:8" "16:4" "24:8" "32:8" "32:12"}; do
  T=${cfg%%:*}; P=${cfg##*:}
  BPG_PRODUCERS=$P timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --threads $T --no-cpu-baseline > gpurun_out/sweep_t${T}_p${P}.json 2> gpurun_out/sweep_t${T}_p${P}.err
done
echo done
