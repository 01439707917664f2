# round-4 GPU step: kernel-trace profile of the final bench command, then local through the batch server vs stock
set -o pipefail
BENCH_ARGS="--no-cpu-baseline" bash scripts/gpu_r04.sh benchprof r04ag || exit 1
K=32 WARM=8 SARGS=--local READS=200000 bash scripts/gpu_r04.sh batch r04ag_local "16"
