#!/bin/bash
# Round 6, call d: smoke + whole GPU suite on the batched power tables /
# draw reduction / tail-weight fills (one launch per lockstep step instead of
# per proof, no upload copies), then A/B of the round-5 build against it.
set -o pipefail
mkdir -p gpurun_out
R=r06d
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1 &&
LIBS="r05:$V/libbpg_r05.so head:" bash scripts/ab_lib.sh ${R} 2 --steps 5 --warmup 2 --no-cpu-baseline --isolated-proofs 0
echo "rc=$?"
