#!/bin/bash
# r03ae: the paired step's host gap -- device memory pool kept (release threshold max,
# BT2G_POOL_KEEP=1) vs the driver default, and with a device-wide sync per step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03ae
mkdir -p $O
B="bench.py --mode paired --no-cpu-baseline --server-sample 0"
BT2G_POOL_KEEP=1 timeout -k 10 600 python -u $B > $O/paired_keep.json 2> $O/paired_keep.log || exit 1
timeout -k 10 600 python -u $B > $O/paired_nokeep.json 2> $O/paired_nokeep.log || exit 1
BT2G_BENCH_TIMING=1 timeout -k 10 600 python -u $B > $O/paired_t.json 2> $O/paired_t.log || exit 1
echo done
