# round-4 GPU step: PMC passes of the batch server's kernels, then the kernel-trace profile of the bench command
set -o pipefail
bash scripts/gpu_r04.sh benchpmc r04x || exit 1
BENCH_ARGS="--no-cpu-baseline" bash scripts/gpu_r04.sh benchprof r04x
