#!/bin/bash
# PMC passes for the roofline (one counter group per pass, kernel-trace only,
# never combined with other trace domains): HBM traffic (FETCH_SIZE, then
# WRITE_SIZE) and the SQ issue/wait counters, over a short bench run at the
# bench's concurrency (THREADS host threads). Only the CSVs go to gpurun_out/.
set -o pipefail
R=${R:-r02c}
ROOTD=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
ARGS=${ARGS:---steps 1 --warmup 1 --threads 8 --batch 32 --no-cpu-baseline}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  rm -rf /tmp/pmc$i
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d /tmp/pmc$i -o run -- \
    python3 $ROOTD/bench.py $ARGS > $ROOTD/gpurun_out/${R}_pmc$i.json 2> $ROOTD/gpurun_out/${R}_pmc$i.err || exit $?
  mkdir -p $ROOTD/gpurun_out/${R}_pmc$i
  for f in $(find /tmp/pmc$i -name '*counter_collection.csv' -o -name '*kernel_trace.csv'); do
    python3 $ROOTD/scripts/pmc_reduce.py "$f" $ROOTD/gpurun_out/${R}_pmc$i/$(basename $f .csv).json
  done
  i=$((i+1))
done
echo done
