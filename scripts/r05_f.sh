#!/bin/bash
# Round 5, call f: smoke + whole GPU suite on the current build (A_I1 split),
# then A/B/C/D of three earlier round-5 commits against it (3 rounds).
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05f}
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_gpu_tests.log 2>&1 &&
LIBS="c71fd7b:$V/libbpg_71fd7bc.so c37a371:$V/libbpg_37a371f.so c4c263c:$V/libbpg_4c263c8.so head:" bash scripts/ab_lib.sh ${R} 3
