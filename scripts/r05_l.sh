#!/bin/bash
# Round 5, call l: smoke, then a four-way A/B in the driver's bench:
#   c0989689  fused first-pass histogram (256-thread digit blocks), scan v1
#   f256      + prefetching column scan (scan v2)
#   e1024     + shuffle scans and 16-bit counts in the scatter, 1024-thread digit blocks
#   c256      + shuffle scans and 16-bit counts in the scatter, 256-thread digit blocks
#   head      + the triple fold's table entries loaded two ops ahead
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05l}
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -v --maxfail=3 --timeout 300 \
    --timeout-method thread > gpurun_out/${R}_parity.log 2>&1 &&
LIBS="c0989689:$V/libbpg_0989689.so f256:$V/libbpg_f256.so e1024:$V/libbpg_e1024.so c256:$V/libbpg_c256.so head:" bash scripts/ab_lib.sh ${R} 2
