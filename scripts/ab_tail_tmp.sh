set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  for t in 4096 512; do
    timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --isolated-proofs 0 --ipp-tail $t > gpurun_out/r06t_t${t}_$i.json 2> gpurun_out/r06t_t${t}_$i.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r06t_t${t}_$i.json')); g=d['gpu_telemetry']; print('tail %-5s run $i  %.2f M constraints/s  %.1f ms/step  sclk %s MHz  power %s W' % ('$t', d['value']/1e6, d['ms_per_step'], g['sclk_mhz']['mean'], g['power_w']['mean']))" >> gpurun_out/r06t_ab.txt
  done
done
cat gpurun_out/r06t_ab.txt
