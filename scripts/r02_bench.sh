#!/bin/bash
# Round-2 bench pass: the driver's own command (steps 20, warmup 5), then the
# default-thread-count bench under rocprofv3 kernel tracing, first without and
# then with the bench's own HIP-event bracketing (round 1 saw a profiler
# SIGSEGV at 16 host threads). Raw profiler databases stay in /tmp; only the
# kernel tables (scripts/prof_summary.py) go to gpurun_out/.
set -o pipefail
R=${R:-r02b}
mkdir -p gpurun_out
ROOTD=$(pwd)
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
fi
cd /tmp && export TMPDIR=/tmp
for live in ${LIVE:-0 1}; do
  rm -rf /tmp/prof_$live
  BENCH_LIVE_TIMING=$live timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/prof_$live -o run -- \
    python3 $ROOTD/bench.py --steps 2 --warmup 1 --no-cpu-baseline ${PROF_ARGS:-} \
    > $ROOTD/gpurun_out/${R}_prof_live$live.json 2> $ROOTD/gpurun_out/${R}_prof_live$live.err
  rc=$?
  db=$(find /tmp/prof_$live -name '*.db' -print -quit)
  [ -n "$db" ] && python3 $ROOTD/scripts/prof_summary.py "$db" $ROOTD/gpurun_out/${R}_prof_live$live.md
  echo "live=$live rc=$rc" >> $ROOTD/gpurun_out/${R}_prof_rc.txt
  [ $rc -ne 0 ] && exit $rc
done
echo done
