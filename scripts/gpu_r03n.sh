#!/bin/bash
# r03n (re-entry): state of the drop-in after c7dbd43 at 3.1 Gbp: SAM parity with the
# speculative-DP verify on, then 2048 / 4096 workers, prefetch off A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03n
mkdir -p $O
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 60 > $O/prof_$tag.txt
}
BT2G_SPEC_VERIFY=1 run g2048v 2048 --reads 100000 --warmup-chunks 4 || exit 1
run g2048 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
run g4096 4096 --reads 400000 --warmup-chunks 12 --skip-stock || exit 1
BT2G_SPEC=0 run g2048nospec 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
echo done
