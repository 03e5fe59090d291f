set -o pipefail
V=$PWD/bulletproof-gadgets_amd/variants
LIBS="r05:$V/libbpg_r05.so final:" bash scripts/ab_lib.sh r06zz_abab2 3 --gpus 1 --steps 12 --warmup 3 --no-cpu-baseline --isolated-proofs 0
