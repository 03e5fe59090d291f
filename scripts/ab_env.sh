#!/bin/bash
# A/B of environment settings for the in-tree build within one gpurun call,
# alternating: ENVS="name:VAR=value,VAR=value name:..." (":" alone = as is)
#   scripts/ab_env.sh <tag> [rounds] [bench args]
set -o pipefail
mkdir -p gpurun_out
T=${1:?tag}; N=${2:-2}; shift 2 || true
ARGS=${*:---steps 5 --warmup 2 --no-cpu-baseline}
for i in $(seq 1 $N); do
  for v in $ENVS; do
    name=${v%%:*}; kv=${v#*:}
    env $(echo "$kv" | tr ',' ' ') timeout -k 10 400 python3 bench.py $ARGS > gpurun_out/${T}_${name}_$i.json 2> gpurun_out/${T}_${name}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/${T}_${name}_$i.json')); print('%-10s run %d  %.2f M constraints/s  %.1f ms/step  hw_queues %s' % ('$name', $i, d['value']/1e6, d['ms_per_step'], d.get('pipeline', {}).get('hw_queues')))" >> gpurun_out/${T}_ab.txt
  done
done
cat gpurun_out/${T}_ab.txt
