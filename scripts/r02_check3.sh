#!/bin/bash
# Parity (fixtures, strategies, full size), the default bench line, and the
# distinct-statement end-to-end line (bench.py --mode statements).
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02t}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${R}_parity.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
timeout -k 10 400 python bench.py --mode statements --steps 2 --warmup 1 --threads 16 --batch 32 > gpurun_out/${R}_statements.json 2> gpurun_out/${R}_statements.err || exit $?
echo done
