#!/bin/bash
# Round 6, call c: robustness + statements tests on the admission fix, then
# an environment A/B of the IPP tail threshold (4096 default vs 32768) and of
# proofs in flight on the no-comb-table path (24 vs 40).
set -o pipefail
mkdir -p gpurun_out
R=r06c
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_robustness.py tests/test_gpu_statements.py -m gpu -v -x --timeout 240 --timeout-method thread > gpurun_out/${R}_robust.log 2>&1 &&
ENVS="base: tail32k:" bash -c 'for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --isolated-proofs 0 > gpurun_out/'${R}'_base_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --isolated-proofs 0 --ipp-tail 32768 > gpurun_out/'${R}'_tail32k_$i.json 2>/dev/null || exit 1
done' &&
timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --isolated-proofs 0 --fold-tables 0 > gpurun_out/${R}_nt24.json 2>/dev/null &&
timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --isolated-proofs 0 --fold-tables 0 --max-inflight 40 --threads 18 > gpurun_out/${R}_nt40.json 2>/dev/null
echo "rc=$?"
