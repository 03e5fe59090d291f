#!/bin/bash
# PMC passes, the sharded latency mode (2 ranks sharing the GPU over gloo),
# then the full-size single-core CPU baseline (no GPU).
set -o pipefail
mkdir -p gpurun_out
ROOTD=$(pwd)
R=r02c bash scripts/r02_pmc.sh || exit $?
cd $ROOTD
timeout -k 10 300 python bench.py --mode latency --steps 5 --warmup 1 > gpurun_out/r02c_latency1.json 2> gpurun_out/r02c_latency1.err || exit $?
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --mode latency --steps 5 --warmup 1 \
  > gpurun_out/r02c_latency2.json 2> gpurun_out/r02c_latency2.err || exit $?
timeout -k 10 900 python -u scripts/cpu_baseline_full.py 5 > gpurun_out/r02c_cpu_full.json 2> gpurun_out/r02c_cpu_full.err || exit $?
echo done
