#!/bin/bash
# End-of-round check on a fresh box: smoke, the whole -m gpu suite, the
# driver's bench command, the 8-thread bench under rocprofv3 (kernel table +
# occupancy timeline; the default 24 threads crash the profiler, DESIGN.md
# (d)), and the PMC passes of the current build. Every GPU step has its own
# time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02x}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
R=${R}_t8 ARGS='--threads 8' bash scripts/r02_trace.sh || exit $?
R=${R} ARGS="${PMC_ARGS:---steps 1 --warmup 1 --threads 8 --batch 32 --no-cpu-baseline}" bash scripts/r02_pmc.sh || exit $?
echo done
