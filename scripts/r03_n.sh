#!/bin/bash
# Round 3, call n: the refactored triple fold (table build and Straus chain as
# device functions) through the parity / full-size tests, then the secondary
# bench modes (verify sample proofs made on 4 threads).
set -o pipefail
R=${R:-r03n}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_scale.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/${R}_verify.json 2> gpurun_out/${R}_verify.err || exit $?
timeout -k 10 300 python bench.py --mode verify-sharded --steps 20 --warmup 3 > gpurun_out/${R}_verify_sharded.json 2> gpurun_out/${R}_verify_sharded.err || exit $?
timeout -k 10 300 python bench.py --mode latency --steps 5 --warmup 1 > gpurun_out/${R}_latency.json 2> gpurun_out/${R}_latency.err || exit $?
timeout -k 10 600 python bench.py --mode statements --steps 2 --warmup 1 > gpurun_out/${R}_statements.json 2> gpurun_out/${R}_statements.err || exit $?
echo done
