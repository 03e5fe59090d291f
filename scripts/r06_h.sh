#!/bin/bash
# Round 6, call h: the prover's generator jobs negate in registers (own
# kernel instantiation k_rbk_pass<true, 1, 2>) and the fused small-row kernel
# at two live points (174 VGPRs): smoke + whole GPU suite, then ABAB of the
# call-f build against it.
set -o pipefail
mkdir -p gpurun_out
R=r06h
V=$PWD/bulletproof-gadgets_amd/variants
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1 &&
LIBS="f:$V/libbpg_f.so head:" bash scripts/ab_lib.sh ${R} 3 --steps 5 --warmup 2 --no-cpu-baseline --isolated-proofs 0
echo "rc=$?"
