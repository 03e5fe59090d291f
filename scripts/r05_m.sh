#!/bin/bash
# Round 5, call m: smoke, then A/B in the driver's bench of
#   c0989689  fused first-pass histogram, column scan v1 (the r05i build)
#   noscat    + device gather of the equal-scalar split at prepare
#   head      + shuffle scans and 16-bit counts in the sort scatter
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05m}
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
LIBS="c0989689:$V/libbpg_0989689.so noscat:$V/libbpg_h_noscat.so head:" bash scripts/ab_lib.sh ${R} 3
