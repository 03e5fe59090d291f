#!/bin/bash
# Round-4 record after the statements lockstep and the batched per-round
# scalar kernels: smoke, the whole GPU suite, the statements layouts on one
# box (8 threads x 1 statement, 5 x 4, and 6 x 4, which the HBM admission must
# cut back), then the driver's bench command.
set -o pipefail
mkdir -p gpurun_out
R=${1:-r04u}
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 &&
timeout -k 10 720 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread \
    > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
for cl in 8:1 5:4 6:4; do
  c=${cl%:*}; l=${cl#*:}
  timeout -k 10 400 python bench.py --mode statements --steps 2 --warmup 1 --consumers $c --stmt-lockstep $l \
      > gpurun_out/${R}_stmts_c${c}l$l.json 2> gpurun_out/${R}_stmts_c${c}l$l.err || exit $?
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
echo "rc=$?"
