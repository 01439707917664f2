# round-4 GPU step: paired with the decision plane + workgroup walk for mate searches (SAM vs stock), and without
set -o pipefail
export K=32 WARM=8 MODE=paired READS=200000
BT2G_DEC_RATIO=6 BT2G_BT_WG_LDS=1 bash scripts/gpu_r04.sh batch r04ad_wide "16" || exit 1
SKIP=--skip-stock bash scripts/gpu_r04.sh batch r04ad "16"
