#!/bin/bash
# A/B: the MSM run reduction in chunks of 32 entries per thread with
# 128-thread blocks (variants/libbpg_t32.so: pass 1 leaves E0/16 slots, the
# merges shrink 16x per pass) against 16 x 256 (default); parity subset on the
# variant first.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04aa}
V=$PWD/bulletproof-gadgets_amd/variants/libbpg_t32.so
BPG_LIB_PATH=$V timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -k "msm or fixture_bit_exact or batch" > gpurun_out/${T}_t32_parity.log 2>&1 || exit $?
for v in default t32 default t32; do
  L=; [ $v = t32 ] && L=$V
  BPG_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_ab_${v}_$SECONDS.json 2> gpurun_out/${T}_ab_${v}.err || exit $?
done
echo done
