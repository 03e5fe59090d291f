#!/bin/bash
# Round 6, call f: small MSM rows spread over all 256 row-kernel threads
# (segments of half / 256 buckets): smoke + whole GPU suite, then A/B of the
# call-e build (segments of 8 buckets) against it.
set -o pipefail
mkdir -p gpurun_out
R=r06f
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1 &&
LIBS="e:$V/libbpg_e.so head:" bash scripts/ab_lib.sh ${R} 2 --steps 5 --warmup 2 --no-cpu-baseline --isolated-proofs 0
echo "rc=$?"
