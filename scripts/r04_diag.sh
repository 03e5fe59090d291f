#!/bin/bash
# Parity diagnostic: the whole device parity module, no -x.
set -o pipefail
mkdir -p gpurun_out
R=${1:-r04i}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/${R}_diag.log 2>&1
echo "pytest rc=$?" >> gpurun_out/${R}_diag.log
