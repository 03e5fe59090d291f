#!/bin/bash
# Batch verification chunk size: 192 proofs over 24 threads (chunks of 8, the
# bench default), 384 over 24 (16), 384 over 12 (32), 384 over 6 (64).
set -o pipefail
mkdir -p gpurun_out
R=${1:-r04y}
for tb in 24:192 24:384 12:384 6:384; do
  t=${tb%:*}; b=${tb#*:}
  timeout -k 10 300 python bench.py --mode verify --steps 3 --warmup 1 --threads $t --batch $b \
      > gpurun_out/${R}_verify_t${t}b$b.json 2> gpurun_out/${R}_verify_t${t}b$b.err || exit $?
done
echo done
