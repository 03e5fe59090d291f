#!/bin/bash
# Which launch configuration crashes rocprofv3 --kernel-trace: the default
# build with round triples off, and a build with 12 MSM segments (smaller
# by-value segment table) with triples off. Each run is short; the profiler
# databases stay in /tmp.
ROOTD=$(pwd)
R=${R:-r02n}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in default s12; do
  if [ $v = s12 ]; then export BPG_LIB_PATH=$ROOTD/bulletproof-gadgets_amd/variants/libbpg_s12.so; else unset BPG_LIB_PATH; fi
  rm -rf /tmp/pc_$v
  BPG_FOLD_TRIPLES=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pc_$v -o run -- python3 $ROOTD/bench.py --steps 1 --warmup 1 --batch 32 --no-cpu-baseline > $ROOTD/gpurun_out/${R}_$v.json 2> $ROOTD/gpurun_out/${R}_$v.err
  echo "$v rc=$?" >> $ROOTD/gpurun_out/${R}_rc.txt
done
echo done
