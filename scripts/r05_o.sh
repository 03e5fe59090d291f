#!/bin/bash
# Round 5, call o: hardware queues per process in the driver's bench
# (the bench raises HIP's default 4 to 16; does a 17th stream share a queue?)
set -o pipefail
mkdir -p gpurun_out
R=${R:-r05o}
ENVS="q16:GPU_MAX_HW_QUEUES=16 q20:GPU_MAX_HW_QUEUES=20 q24:GPU_MAX_HW_QUEUES=24" bash scripts/ab_env.sh ${R} 2
