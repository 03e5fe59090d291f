#!/bin/bash
# End-of-round check A on a fresh box: smoke, the whole -m gpu suite and the
# driver's bench command. Every GPU step has its own limit; the first
# failure ends the script.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r03z}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
echo done
