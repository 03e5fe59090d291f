#!/bin/bash
# Round 6, call i: the final build's statements mode (prepare keeps its
# witness buffers again, up to 32 MB each), then the hosts records: the
# two-rank launcher run and the rank pinned to 2, 3 and 4 CPUs.
set -o pipefail
mkdir -p gpurun_out
R=r06zz
timeout -k 10 600 python bench.py --mode statements --steps 2 --warmup 1 > gpurun_out/${R}_statements2.json 2> gpurun_out/${R}_statements2.err &&
R=${R} bash scripts/final_check.sh hosts
echo "rc=$?"
