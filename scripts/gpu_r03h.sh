#!/bin/bash
# r03h: drop-in vs stock server on the 3.1 Gbp hg38-like index (north-star config), current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03h
mkdir -p $O
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --top 60 > $O/prof_$tag.txt
  python scripts/prof_symbolize.py $O/samp_$tag.txt --callers-of mprotect --top 12 > $O/mprotect_$tag.txt
}
run g2048 2048 --reads 300000 --warmup-chunks 3 || exit 1
BT2G_ADAPTER_PROF=1 run g2048p 2048 --reads 200000 --warmup-chunks 2 --skip-stock || exit 1
echo done
