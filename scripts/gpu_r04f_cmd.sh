# round-4 GPU step: kernel-trace profile of the bench command without the walk's LDS opt-in (rocprofv3 crashed
# in its own library on the opt-in path, r04ag), then local through the batch server vs stock
set -o pipefail
BT2G_BT_WG_LDS=0 BENCH_ARGS="--no-cpu-baseline" bash scripts/gpu_r04.sh benchprof r04ah || exit 1
K=32 WARM=8 SARGS=--local READS=200000 bash scripts/gpu_r04.sh batch r04ah_local "16"
