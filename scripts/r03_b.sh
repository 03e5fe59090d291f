#!/bin/bash
# Round 3, call b: the new statements test, A/B of the two-level row
# reduction (default) against the one-block-per-row build, the statements
# bench through bpg_prove_statements, then rocprofv3 on the default
# 24-thread bench (last: a profiler crash ends the call).
set -o pipefail
R=${R:-r03b}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_statements.py -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_stmt_test.log 2>&1 || { echo "stmt test rc=$?"; exit 1; }
for v in new old new old; do
  if [ $v = old ]; then export BPG_LIB_PATH=$PWD/bulletproof-gadgets_amd/variants/libbpg_row1.so; else unset BPG_LIB_PATH; fi
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_$v.json 2>> gpurun_out/${R}_ab.err || { echo "ab rc=$?"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${R}_ab_$v.json'));print('$v', d['value'], d['ms_per_step'])" >> gpurun_out/${R}_ab.txt
done
unset BPG_LIB_PATH
timeout -k 10 600 python bench.py --mode statements --steps 2 --warmup 1 > gpurun_out/${R}_statements.json 2> gpurun_out/${R}_statements.err || { echo "statements rc=$?"; exit 1; }
ROOTD=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/${R}_prof -o run -- python3 $ROOTD/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOTD/gpurun_out/${R}_prof_bench.json 2> $ROOTD/gpurun_out/${R}_prof.err
rc=$?
echo "prof rc=$rc" >> $ROOTD/gpurun_out/${R}_prof_rc.txt
cd $ROOTD
if [ $rc = 0 ]; then
  db=$(find /tmp/${R}_prof -name '*.db' -print -quit)
  python3 scripts/prof_summary.py "$db" gpurun_out/${R}_prof_kernels.md > /dev/null
  python3 scripts/timeline.py "$db" 0.35 gpurun_out/${R}_timeline.md 0.92 > /dev/null
fi
echo done
