#!/bin/bash
# Round 5, call g: smoke + whole GPU suite (write-through reduction hand-off),
# then A/B of the release-fence build (2b7edd7) against it.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05g}
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_gpu_tests.log 2>&1 &&
LIBS="c2b7edd:$V/libbpg_2b7edd7.so head:" bash scripts/ab_lib.sh ${R} 3
