# round-4 GPU step: the batch server's read supply (read buffers per connection) and hardware queues
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
K=32 WARM=8 READS=400000 BT2G_KPROF=1 bash scripts/gpu_r04.sh batch r04q "16" || exit 1
SKIP=--skip-stock K=32 WARM=8 READS=400000 BT2G_READAHEAD=65 bash scripts/gpu_r04.sh batch r04q_ra65 "16" || exit 1
SKIP=--skip-stock K=32 WARM=8 READS=400000 BT2G_READAHEAD=65 BT2G_HW_QUEUES=16 bash scripts/gpu_r04.sh batch r04q_ra65hq16 "16" || exit 1
SKIP=--skip-stock K=64 WARM=8 READS=400000 BT2G_READAHEAD=65 bash scripts/gpu_r04.sh batch r04q_ra65k64 "16"
