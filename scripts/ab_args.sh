#!/bin/bash
# A/B of bench arguments on the in-tree library within one gpurun call,
# alternating (ABAB...):
#   VARIANTS="name=extra args;name=extra args" scripts/ab_args.sh <tag> [rounds] [common bench args]
# One bench line per run under gpurun_out/<tag>_<name>_<i>.json and a
# summary table in gpurun_out/<tag>_ab.txt. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
T=${1:?tag}; N=${2:-2}; shift 2 || true
ARGS=${*:---steps 5 --warmup 2 --no-cpu-baseline}
IFS=';' read -ra VS <<< "${VARIANTS:?VARIANTS}"
for i in $(seq 1 $N); do
  for v in "${VS[@]}"; do
    name=${v%%=*}; extra=${v#*=}
    timeout -k 10 400 python3 bench.py $ARGS $extra > gpurun_out/${T}_${name}_$i.json 2> gpurun_out/${T}_${name}_$i.err || exit $?
    python3 -c "import json,sys; d=json.load(open('gpurun_out/${T}_${name}_$i.json')); g=d.get('gpu_telemetry') or {}; print('%-10s run %d  %.2f M constraints/s  %.1f ms/step  latency %.1f ms  sclk %s MHz  power %s W' % ('$name', $i, d['value']/1e6, d['ms_per_step'], d.get('latency_ms_single_proof') or 0, (g.get('sclk_mhz') or {}).get('mean'), (g.get('power_w') or {}).get('mean')))" >> gpurun_out/${T}_ab.txt
  done
done
cat gpurun_out/${T}_ab.txt
