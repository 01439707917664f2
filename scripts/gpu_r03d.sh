#!/bin/bash
# r03d: long warm-up (is the per-fiber cost a start-up transient?), no active GPU wait
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03d
mkdir -p $O
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 500 python -u scripts/dropin_bench.py --genome-mb 200 \
    --k 8 --gpu-workers $w --workdir /tmp/db200 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --top 50 > $O/prof_$tag.txt
  python scripts/prof_symbolize.py $O/samp_$tag.txt --callers-of mprotect --top 10 > $O/mprotect_$tag.txt
}
run f1024 1024 --reads 300000 --warmup-chunks 5 || exit 1
run f4096 4096 --reads 300000 --warmup-chunks 5 --skip-stock || exit 1
run f4096w12 4096 --reads 300000 --warmup-chunks 12 --skip-stock || exit 1
echo done
