# round-4 GPU step: slab pages A/B on one box, then bench
set -o pipefail
export K=32 WARM=8 READS=400000 BT2G_KPROF=1
bash scripts/gpu_r04.sh batch r04z "16" || exit 1
SKIP=--skip-stock BT2G_SLAB_HUGE=0 bash scripts/gpu_r04.sh batch r04z_small "16" || exit 1
unset K WARM READS BT2G_KPROF
bash scripts/gpu_r04.sh bench r04z
