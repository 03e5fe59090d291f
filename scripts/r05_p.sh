#!/bin/bash
# Round 5, call p: smoke + the GPU suite, then A/B of 403b542 against the
# wave-shuffle scalar block reductions (t(x), c_L / c_R, dots, flatten).
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05p}
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_gpu_tests.log 2>&1 &&
LIBS="c403b542:$V/libbpg_403b542.so head:" bash scripts/ab_lib.sh ${R} 3
