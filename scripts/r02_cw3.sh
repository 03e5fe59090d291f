#!/bin/bash
# A/B: MSM pass 1 over cached (folded) bases compiled for 3 waves per SIMD
# (RBK_CWAVES=3: 168 VGPRs, 28 B/lane scratch) vs the default 2, ABAB on one
# box, and the parity tests on the variant library.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab_summary.txt
V=bulletproof-gadgets_amd/variants/libbpg_cw3.so
BPG_LIB_PATH=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02zz_cw3_parity.log 2>&1 || exit $?
STEPS=3 VARIANTS="d1:X=1 cw3a:BPG_LIB_PATH=$V d2:X=1 cw3b:BPG_LIB_PATH=$V" bash scripts/ab.sh || exit $?
echo done
