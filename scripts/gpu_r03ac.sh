#!/bin/bash
# r03ac: batching knobs of the drop-in on the final tree: batch window 200 -> 100 us, carrier
# flush 100 -> 50 us, DP dispatchers 4 -> 6 (scheduling only: no alignment changes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03ac
mkdir -p $O /tmp/db3100
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
}
run base 4096 --reads 400000 --warmup-chunks 12 --dropin-args='--reads-per-batch 4' || exit 1
BT2G_BATCH_WINDOW_US=100 BT2G_FLUSH_US=50 run fast 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 4' || exit 1
BT2G_SEAM_THREADS_sw_dp=6 run dp6 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 4' || exit 1
echo done
