#!/bin/bash
# A/B bench runs: each VARIANTS entry is "name:ENV=VAL[,ENV=VAL]"; one bench
# line per variant under gpurun_out/ab_<name>.json, summary in ab_summary.txt.
set -e
mkdir -p gpurun_out
for v in $VARIANTS; do
  name=${v%%:*}; envs=${v#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 300 python3 bench.py --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err
  echo "$name $(python3 -c "import json; d=json.load(open('gpurun_out/ab_$name.json')); print(d['value'], d['ms_per_step'], d['phase_ms_single_proof']['total_ms'])")" >> gpurun_out/ab_summary.txt
done
echo done
