#!/bin/bash
# Distinct statements end to end through c_prove (parse, synthesis, upload,
# prove) after the host-synthesis speed-up, and batch verification, on the
# final tree. Every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02zz}
timeout -k 10 500 python bench.py --mode statements --steps 2 --warmup 1 --threads 16 --batch 32 > gpurun_out/${R}_statements.json 2> gpurun_out/${R}_statements.err || exit $?
timeout -k 10 400 python bench.py --mode verify > gpurun_out/${R}_verify.json 2> gpurun_out/${R}_verify.err || exit $?
echo done
