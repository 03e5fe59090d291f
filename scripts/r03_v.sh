#!/bin/bash
# Round 3, call v: the consumer layout under the wave-priority default:
# three proofs per consumer step (BPG_LOCKSTEP=3: 8 consumers, 24 in flight)
# and 28 proofs in flight (BPG_MAX_INFLIGHT=28: 7 consumers of four; ~304 of
# the 309 GB of HBM, so it runs last) against the default (6 consumers of
# four). Default bench command shortened to 3 steps. Every GPU step has its
# own limit; the first failure ends the script.
set -o pipefail
R=${R:-r03v}
mkdir -p gpurun_out
run() {
  local v=$1; shift
  env "$@" timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_$v.json 2>> gpurun_out/${R}_ab.err || { echo "ab $v rc=$?"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$v.json'));print('$v', d['value'], d['ms_per_step'], d['hbm_used_gb'], d['roofline']['device_ms_by_kernel'])" >> gpurun_out/${R}_ab.txt
}
run base BPG_NONE=0
run ls3 BPG_LOCKSTEP=3
run base BPG_NONE=0
run ls3 BPG_LOCKSTEP=3
run if28 BPG_MAX_INFLIGHT=28
run if28 BPG_MAX_INFLIGHT=28
echo done
