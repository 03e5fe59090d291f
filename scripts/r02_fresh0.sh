#!/bin/bash
# Pass-1 entry-0 conversion (RBK_FRESH0): smoke and the whole -m gpu suite on
# the new default build, then an A/B against the RBK_FRESH0=0 variant (the previous code) built
# from the same tree (ABAB, same box), then the driver's bench command.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02zz}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${R}_gpu_tests.log 2>&1 || exit $?
STEPS=3 VARIANTS="off1:BPG_LIB_PATH=bulletproof-gadgets_amd/variants/libbpg_base.so on1:X=1 off2:BPG_LIB_PATH=bulletproof-gadgets_amd/variants/libbpg_base.so on2:X=1" bash scripts/ab.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err || exit $?
echo done
