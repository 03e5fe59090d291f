#!/bin/bash
# Distinct statements proved up to four at a time in lockstep, consumers
# admitted by HBM: smoke, the whole GPU suite, the statements bench at the
# default 5 device threads and at 6 (more than HBM admits), then the verify
# bench with 16-proof chunks (384 proofs over 24 threads) and 32-proof chunks
# (12 threads).
set -o pipefail
mkdir -p gpurun_out
R=${1:-r04t}
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
for c in 5 6; do
  timeout -k 10 400 python bench.py --mode statements --steps 2 --warmup 1 --consumers $c > gpurun_out/${R}_stmts_c$c.json 2> gpurun_out/${R}_stmts_c$c.err || exit $?
done
timeout -k 10 300 python bench.py --mode verify --steps 3 --warmup 1 --batch 384 > gpurun_out/${R}_verify_b384.json 2> gpurun_out/${R}_verify_b384.err &&
timeout -k 10 300 python bench.py --mode verify --steps 3 --warmup 1 --threads 12 --batch 384 > gpurun_out/${R}_verify_t12.json 2> gpurun_out/${R}_verify_t12.err
echo "rc=$?"
