#!/bin/bash
# Re-check after the container was re-created: smoke, the whole -m gpu
# suite and the driver's bench command on the rebuilt tree. Every GPU step
# has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02zz}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
echo done
