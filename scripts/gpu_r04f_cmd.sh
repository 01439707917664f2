# round-4 GPU step: two lanes vs one, then bench.py as the driver runs it
set -o pipefail
export K=32 WARM=8 READS=400000 BT2G_KPROF=1
bash scripts/gpu_r04.sh batch r04u_l2 "16" || exit 1
SKIP=--skip-stock BT2G_LANES=1 bash scripts/gpu_r04.sh batch r04u_l1 "16" || exit 1
unset K WARM READS BT2G_KPROF
bash scripts/gpu_r04.sh bench r04u
