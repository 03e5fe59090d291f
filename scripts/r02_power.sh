#!/bin/bash
# Power / clock / activity of the GPU while the default bench runs: is the
# prove throughput bound by the chip's power limit (clock drops under VALU
# load) or by idle issue slots? rocm-smi sampled once a second next to a
# short bench run.
set -o pipefail
R=${R:-r02f}
mkdir -p gpurun_out
( for i in $(seq 1 150); do echo "@ $(date +%s.%N)"; timeout 10 rocm-smi --showpower --showclocks --showuse --showtemp 2>&1 | grep -E "^(GPU|card)" ; sleep 1; done ) > gpurun_out/${R}_smi.log 2>&1 &
SMI=$!
timeout -k 10 400 python3 bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
rc=$?
kill $SMI
timeout 20 rocm-smi --showmaxpower --showclkfrq 2>&1 | head -60 > gpurun_out/${R}_smi_static.log
exit $rc
