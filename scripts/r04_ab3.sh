#!/bin/bash
# A/B: materialised IPP levels converted to affine Niels (variants/libbpg_niels.so,
# parity module first), the RNG slot layout of round 3 (8 per producer + 2
# per consumer, variants/libbpg_oldslots.so), against the in-tree default.
set -o pipefail
mkdir -p gpurun_out
T=${1:-r04o}
VD=$PWD/bulletproof-gadgets_amd/variants
BPG_LIB_PATH=$VD/libbpg_niels.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -k "not hbm_admission" > gpurun_out/${T}_niels_parity.log 2>&1 || exit $?
for v in default niels oldslots default niels; do
  L=; [ $v != default ] && L=$VD/libbpg_$v.so
  BPG_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_ab_${v}_$SECONDS.json 2> gpurun_out/${T}_ab_${v}.err || exit $?
done
echo done
