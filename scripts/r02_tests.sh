#!/bin/bash
# Round-2 GPU test pass: page torch in (the sharded tests start one process
# per rank), then the whole -m gpu suite; logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -c "import torch; print('torch', torch.__version__)" > gpurun_out/${R:-r02}_torch.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${R:-r02}_gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/${R:-r02}_gpu_tests.log
exit $rc
