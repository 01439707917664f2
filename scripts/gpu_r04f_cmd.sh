# round-4 GPU step: DP staging fix (first-pass edit room, doubling arenas), local kernels, bench
set -o pipefail
export K=32 WARM=8 READS=400000 BT2G_KPROF=1
bash scripts/gpu_r04.sh batch r04w "16" || exit 1
SKIP=--skip-stock SARGS=--local READS=200000 bash scripts/gpu_r04.sh batch r04w_local "16" || exit 1
unset K WARM READS BT2G_KPROF
bash scripts/gpu_r04.sh bench r04w
