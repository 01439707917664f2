# round-4 GPU step: paired (mate-search DPs in calls of their own) vs stock, unpaired, bench
set -o pipefail
export K=32 WARM=8
MODE=paired READS=200000 bash scripts/gpu_r04.sh batch r04ab_paired "16" || exit 1
READS=400000 BT2G_KPROF=1 bash scripts/gpu_r04.sh batch r04ab "16" || exit 1
unset K WARM
bash scripts/gpu_r04.sh bench r04ab
