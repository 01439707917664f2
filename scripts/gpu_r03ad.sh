#!/bin/bash
# r03ad: the paired step with and without BT2G_BENCH_TIMING (a device-wide sync at step start)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03ad
mkdir -p $O
timeout -k 10 600 python -u bench.py --mode paired --no-cpu-baseline --server-sample 0 > $O/paired.json 2> $O/paired.log || exit 1
BT2G_BENCH_TIMING=1 timeout -k 10 600 python -u bench.py --mode paired --no-cpu-baseline --server-sample 0 > $O/paired_t.json 2> $O/paired_t.log || exit 1
echo done
