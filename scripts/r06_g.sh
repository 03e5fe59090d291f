#!/bin/bash
# Round 6, call g: generator MSM jobs negating in registers (one 256 MB
# gather set instead of 512 MB with the negated copies; the chip runs
# power-limited at ~2.12 GHz, so fewer bytes moved may buy clock): parity of
# the variant on the fixture and strategy tests, then ABAB against the head.
set -o pipefail
mkdir -p gpurun_out
R=r06g
V=$PWD/bulletproof-gadgets_amd/variants
BPG_LIB_PATH=$V/libbpg_neg.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${R}_neg_parity.log 2>&1 &&
LIBS="head: neg:$V/libbpg_neg.so" bash scripts/ab_lib.sh ${R} 3 --steps 5 --warmup 2 --no-cpu-baseline --isolated-proofs 0
echo "rc=$?"
