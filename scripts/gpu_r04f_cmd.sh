# round-4 GPU step: DP service workers x hardware queues (read-ahead 65)
set -o pipefail
O=gpurun_out/r04r; mkdir -p $O
export K=32 WARM=8 READS=400000 BT2G_READAHEAD=65 BT2G_KPROF=1
BT2G_HW_QUEUES=16 BT2G_DP_WORKERS=6 bash scripts/gpu_r04.sh batch r04r_hq16dp6 "16" || exit 1
SKIP=--skip-stock BT2G_HW_QUEUES=32 BT2G_DP_WORKERS=6 bash scripts/gpu_r04.sh batch r04r_hq32dp6 "16" || exit 1
SKIP=--skip-stock BT2G_HW_QUEUES=32 BT2G_DP_WORKERS=8 BT2G_SVC_WORKERS=3 bash scripts/gpu_r04.sh batch r04r_hq32dp8s3 "16" || exit 1
SKIP=--skip-stock BT2G_HW_QUEUES=16 BT2G_DP_WORKERS=4 BT2G_BATCH_SLOTS=4096 bash scripts/gpu_r04.sh batch r04r_hq16dp4sl4k "16"
