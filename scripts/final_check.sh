#!/bin/bash
# End-of-round records, two gpurun calls:
#   R=<tag> bash scripts/final_check.sh prof    the default bench command under
#       rocprofv3 --kernel-trace --stats (kernel table + occupancy timeline;
#       the bench's own HIP-event bracketing on), then the PMC passes of the
#       same build (one counter group per pass, kernel trace only) over the
#       default layout at 48 proofs per step, reduced to a per-kernel table
#       that pairs each kernel's HBM bytes with its algorithmic bytes from the
#       same run; and `bench.py --mode isolated` (one consumer stream) under
#       the same trace: the kernels' own chip time, the roofline's basis
#   R=<tag> bash scripts/final_check.sh abab    the round-4 and round-5 driver-measured
#       builds (variants/libbpg_r04.so, _r05.so) against the final build, ABAB
#   R=<tag> bash scripts/final_check.sh modes   the driver's bench command, then
#       the secondary modes (verify, verify-sharded, latency, statements)
#   R=<tag> bash scripts/final_check.sh hosts   the --gpus launcher with two
#       self-spawned ranks sharing the one GPU over gloo (RCCL refuses two
#       ranks on one device), config 4; then the rank pinned to 2, 3 and 4
#       CPUs (an 8-GPU node's per-rank share)
set -o pipefail
mkdir -p gpurun_out
R=${R:?tag}
ROOTD=$(pwd)
if [ "$1" = abab ]; then
  # the previous driver-measured builds against the final one on one box,
  # alternating, with the driver's command (clock and power in every line)
  V=$ROOTD/bulletproof-gadgets_amd/variants
  LIBS="r04:$V/libbpg_r04.so r05:$V/libbpg_r05.so final:" bash scripts/ab_lib.sh ${R}_abab 2 --gpus 1 --steps 12 --warmup 3 --no-cpu-baseline --isolated-proofs 0 || exit $?
elif [ "$1" = prof ]; then
  (cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/${R}_prof && \
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/${R}_prof -o run -- python3 $ROOTD/bench.py --steps 3 --warmup 1 --no-cpu-baseline --isolated-proofs 0 > $ROOTD/gpurun_out/${R}_profdefault_bench.json 2> $ROOTD/gpurun_out/${R}_profdefault.err) || exit $?
  db=$(find /tmp/${R}_prof -name '*.db' -print -quit)
  python3 scripts/prof_summary.py "$db" gpurun_out/${R}_profdefault_kernels.md > /dev/null || exit $?
  python3 scripts/timeline.py "$db" 0.35 gpurun_out/${R}_timeline_default.md 0.92 > /dev/null || exit $?
  # the isolated leg alone (one consumer stream): the per-kernel averages the
  # bench line's roofline.frac uses (avg_launch_ms) must agree with this table
  (cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/${R}_iso && \
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/${R}_iso -o run -- python3 $ROOTD/bench.py --mode isolated --warmup 1 > $ROOTD/gpurun_out/${R}_isolated_bench.json 2> $ROOTD/gpurun_out/${R}_isolated.err) || exit $?
  db=$(find /tmp/${R}_iso -name '*.db' -print -quit)
  python3 scripts/prof_summary.py "$db" gpurun_out/${R}_isolated_kernels.md > /dev/null || exit $?
  R=${R} ARGS="--steps 1 --warmup 1 --batch 48 --no-cpu-baseline --isolated-proofs 0" bash scripts/pmc_passes.sh || exit $?
  python3 scripts/pmc_table.py gpurun_out/${R} gpurun_out/${R}_pmc.json > gpurun_out/${R}_pmc_table.md || exit $?
elif [ "$1" = modes ]; then
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
  timeout -k 10 300 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/${R}_verify.json 2> gpurun_out/${R}_verify.err || exit $?
  timeout -k 10 300 python bench.py --mode verify-sharded --steps 20 --warmup 3 > gpurun_out/${R}_verify_sharded.json 2> gpurun_out/${R}_verify_sharded.err || exit $?
  timeout -k 10 300 python bench.py --mode latency --steps 5 --warmup 1 > gpurun_out/${R}_latency.json 2> gpurun_out/${R}_latency.err || exit $?
  timeout -k 10 600 python bench.py --mode statements --steps 2 --warmup 1 > gpurun_out/${R}_statements.json 2> gpurun_out/${R}_statements.err || exit $?
else   # hosts: the two-rank launcher run and the per-rank CPU shares
  BENCH_DIST_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --config 4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${R}_bench_2ranks_shared_gpu.json 2> gpurun_out/${R}_bench_2ranks.err || exit $?
  # the per-rank CPU share of an 8-GPU node: the rank pinned to 2, 3 and 4 CPUs
  for c in 2 3 4; do
    timeout -k 10 400 python bench.py --steps 8 --warmup 2 --cpus $c --no-cpu-baseline --isolated-proofs 0 > gpurun_out/${R}_cpus$c.json 2> gpurun_out/${R}_cpus$c.err || exit $?
  done
fi
echo done
