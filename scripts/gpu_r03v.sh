#!/bin/bash
# r03v: per-connection read-ahead depth under fibers (each buffer = a PatternSourcePerThread of
# 2 x batch Reads built and freed per connection; default nthreads + 1 = 4097 per connection)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03v
mkdir -p $O /tmp/db3100
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_MUTEX_PROF=$PWD/$O/mx_$tag.txt BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 40 > $O/prof_$tag.txt
}
BT2G_READAHEAD=600 run g4096ra600 4096 --reads 400000 --warmup-chunks 12 --dropin-args='--reads-per-batch 4' || exit 1
BT2G_READAHEAD=1200 run g4096ra1200 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 4' || exit 1
run g4096 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 4' || exit 1
echo done
