#!/bin/bash
# GPU-box check: microbenchmarks (optional), parity tests, bench line,
# rocprofv3 kernel stats. Every GPU step has its own time limit; the first
# failure ends the script.
set -e
mkdir -p gpurun_out
R=${ROUND:-r01}
if [ "${MICRO:-0}" = 1 ]; then
  (cd bulletproof-gadgets_amd && timeout -k 10 120 bin/comb_bench && timeout -k 10 120 bin/fold_bench_w2) > gpurun_out/${R}_micro.log 2>&1
fi
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/${R}_gpu_tests.log 2>&1
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
fi
if [ "${PROF:-1}" = 1 ]; then
  ROOTD=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  # the bench's own default command under the profiler (rocpd output; the
  # CSV writer of rocprofv3 crashed with 16 host threads)
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/${R}_prof -o run -- python3 $ROOTD/bench.py ${PROF_ARGS:-} > $ROOTD/gpurun_out/${R}_prof_bench.json 2> $ROOTD/gpurun_out/${R}_prof.err
  cd $ROOTD
fi
echo done
