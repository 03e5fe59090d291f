#!/bin/bash
# A/B: IPP tail threshold 2048 / 4096 (default) / 8192 lanes with the
# round-4 prover (folded levels as Niels points), alternated twice.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04ac}
for i in 1 2; do
  for t in 4096 2048 8192; do
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --ipp-tail $t > gpurun_out/${T}_tail${t}_$i.json 2> gpurun_out/${T}_tail${t}_$i.err || exit $?
  done
done
echo done
