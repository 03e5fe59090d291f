#!/bin/bash
# MSM window-width sweep: fold_bench's MSM jobs at c = lg(points) - bias.
set -e
mkdir -p gpurun_out
cd bulletproof-gadgets_amd
for b in 3 4 5; do
  echo "bias $b"
  BPG_MSM_C_BIAS=$b timeout -k 10 120 bin/fold_bench_w2 | grep msm
done > ../gpurun_out/msm_bias.log 2>&1
