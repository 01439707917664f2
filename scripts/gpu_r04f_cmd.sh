# round-4 GPU step: bench.py with 16 hardware queues again, then paired through the batch server
set -o pipefail
bash scripts/gpu_r04.sh bench r04af || exit 1
K=32 WARM=8 MODE=paired READS=200000 SKIP=--skip-stock bash scripts/gpu_r04.sh batch r04af_paired "16"
