#!/bin/bash
# Round 5, call t: smoke + the GPU suite, then A/B of 4e0aef6 against the
# A_I1 split gathered at commit time (a statement in flight holds only the
# lane indices) and prepared buffers allocated exactly: statements mode, then
# the driver's bench.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05t}
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_gpu_tests.log 2>&1 &&
LIBS="c4e0aef6:$V/libbpg_4e0aef6.so head:" bash scripts/ab_lib.sh ${R}_stmts 2 --mode statements --steps 2 --warmup 1 --no-cpu-baseline &&
LIBS="c4e0aef6:$V/libbpg_4e0aef6.so head:" bash scripts/ab_lib.sh ${R} 2
