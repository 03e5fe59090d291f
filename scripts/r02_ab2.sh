#!/bin/bash
# Parity of the current build (fixtures, strategies, full size, MSM edge
# cases), A/B bench lines vs the variants in AB, then the distinct-statement
# line.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02u}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${R}_parity.log 2>&1 || exit $?
SKIP_PARITY=1 R=$R bash scripts/r02_ab.sh || exit $?
timeout -k 10 400 python bench.py --mode statements --steps 2 --warmup 1 --threads 16 --batch 32 > gpurun_out/${R}_statements.json 2> gpurun_out/${R}_statements.err
echo "statements rc=$?" >> gpurun_out/${R}_ab_summary.txt
echo done
