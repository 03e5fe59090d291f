#!/bin/bash
# New GPU tests (reference matrix, CLI, robustness, sharded), the VALU-rate
# microbenchmarks behind the roofline's fe_mul peak, the latency mode at 2
# ranks sharing the GPU (gloo), and the full-size single-core CPU baseline.
set -o pipefail
mkdir -p gpurun_out
R=r02d
timeout -k 10 240 python -c "import torch" || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_reference_matrix.py tests/test_gpu_robustness.py tests/test_gpu_sharded.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
(cd bulletproof-gadgets_amd && timeout -k 10 120 bin/isa_rates && timeout -k 10 120 bin/fe_variants) > gpurun_out/${R}_valu_micro.log 2>&1 || exit $?
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --mode latency --steps 5 --warmup 1 \
  > gpurun_out/${R}_latency2.json 2> gpurun_out/${R}_latency2.err || exit $?
timeout -k 10 900 python -u scripts/cpu_baseline_full.py 5 > gpurun_out/${R}_cpu_full.json 2> gpurun_out/${R}_cpu_full.err || exit $?
echo done
