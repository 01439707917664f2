# round-4 GPU step: batch server host phases of the DP call (KPROF), then paired and local vs stock
set -o pipefail
export K=32 WARM=8 READS=400000
BT2G_KPROF=1 bash scripts/gpu_r04.sh batch r04v "16" || exit 1
MODE=paired READS=200000 bash scripts/gpu_r04.sh batch r04v_paired "16" || exit 1
SARGS=--local bash scripts/gpu_r04.sh batch r04v_local "16"
