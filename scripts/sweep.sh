#!/bin/bash
# Throughput sweep on the GPU box: RNG rate per thread, then bench at several
# host-thread / producer / hardware-queue splits. CFGS entries are
# threads:producers[:hw_queues]. Output under gpurun_out/sweep_*.
set -e
mkdir -p gpurun_out
echo "cpus: $(nproc) affinity: $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')" > gpurun_out/sweep_env.txt
lscpu | grep -E "Model name|Socket|Core|Thread" >> gpurun_out/sweep_env.txt || true
for cfg in ${CFGS:-"16:8" "16:4" "24:8" "32:8" "32:12"}; do
  IFS=: read T P Q <<< "$cfg"
  Q=${Q:-4}
  GPU_MAX_HW_QUEUES=$Q BPG_PRODUCERS=$P timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --threads $T ${BATCH:+--batch $BATCH} --no-cpu-baseline > gpurun_out/sweep_t${T}_p${P}_q${Q}.json 2> gpurun_out/sweep_t${T}_p${P}_q${Q}.err
  echo "$cfg $(python3 -c "import json; d=json.load(open('gpurun_out/sweep_t${T}_p${P}_q${Q}.json')); print(d['value'], d['ms_per_step'])")" >> gpurun_out/sweep_summary.txt
done
echo done
