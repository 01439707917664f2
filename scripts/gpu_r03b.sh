#!/bin/bash
# r03b: fiber drop-in after the allocator / carrier-count fixes (200 Mbp, 200 k reads)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03b
mkdir -p $O
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 400 python -u scripts/dropin_bench.py --genome-mb 200 --reads 200000 \
    --k 8 --gpu-workers $w --workdir /tmp/db200 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --top 70 > $O/prof_$tag.txt
}
run f1024 1024 || exit 1
run f4096 4096 --skip-stock || exit 1
BT2G_BATCH_WINDOW_US=50 run f4096w50 4096 --skip-stock || exit 1
echo done
