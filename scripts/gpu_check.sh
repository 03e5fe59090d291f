#!/bin/bash
# GPU-box check: parity tests, bench line, rocprofv3 kernel stats.
set -e
mkdir -p gpurun_out
R=${ROUND:-r01}
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/${R}_gpu_tests.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
if [ "${PROF:-1}" = 1 ]; then
  ROOTD=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $ROOTD/gpurun_out/${R}_prof -o run -- python3 $ROOTD/bench.py --steps 2 --threads ${PROF_THREADS:-2} --batch ${PROF_BATCH:-4} --no-cpu-baseline > $ROOTD/gpurun_out/${R}_prof_bench.json 2> $ROOTD/gpurun_out/${R}_prof.err
  cd $ROOTD
fi
echo done
