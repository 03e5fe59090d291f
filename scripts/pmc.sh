#!/bin/bash
# PMC passes (rocprofv3 --pmc, one counter group per pass, kernel-trace only)
# over a small bench run; per-dispatch counters land in gpurun_out/${R}_pmc*/.
set -e
R=${ROUND:-r01}
ROOTD=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"; do
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $ROOTD/gpurun_out/${R}_pmc$i -o run -- python3 $ROOTD/bench.py --steps 1 --warmup 1 --threads 1 --batch 1 --no-cpu-baseline > $ROOTD/gpurun_out/${R}_pmc$i.json 2> $ROOTD/gpurun_out/${R}_pmc$i.err
  i=$((i+1))
done
echo done
