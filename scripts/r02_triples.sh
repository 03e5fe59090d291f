#!/bin/bash
# Round triples: parity of every fold strategy (small fixtures with a low IPP
# tail threshold, full-size goldens on the default path, full-size strategy
# cross-check), then A/B bench lines: default (triples) vs pairs
# (BPG_FOLD_TRIPLES=0), alternating.
set -o pipefail
mkdir -p gpurun_out
R=${R:-r02i}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_scale.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${R}_parity.log 2>&1 || exit $?
for rep in 1 2; do
  for v in default pairs; do
    if [ "$v" = pairs ]; then export BPG_FOLD_TRIPLES=0; else unset BPG_FOLD_TRIPLES; fi
    timeout -k 10 300 python bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > gpurun_out/${R}_ab_${v}_$rep.json 2> gpurun_out/${R}_ab_${v}_$rep.err || exit $?
    echo "$v $rep $(python3 -c "import json; d=json.loads(open('gpurun_out/${R}_ab_${v}_$rep.json').read().strip().splitlines()[-1]); k=d['roofline']['device_ms_by_kernel']; print(d['value'], d['ms_per_step'], d['latency_ms_single_proof'], k.get('ipp_fold2'), k.get('ipp_fold3'), k.get('msm_pass1_cached'))")" >> gpurun_out/${R}_ab_summary.txt
  done
done
unset BPG_FOLD_TRIPLES
echo done
