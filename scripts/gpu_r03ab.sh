#!/bin/bash
# r03ab: slab-backed caching allocator; read-ahead 1025 vs 4097 per connection; prefetch on/off
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03ab
mkdir -p $O /tmp/db3100
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_ALLOC_STATS=$PWD/$O/alloc_$tag.txt BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 40 > $O/prof_$tag.txt
}
BT2G_READAHEAD=1025 run g4096ra1025 4096 --reads 400000 --warmup-chunks 12 --dropin-args='--reads-per-batch 4' || exit 1
run g4096 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 4' || exit 1
BT2G_SEEDPF=0 BT2G_READAHEAD=1025 run g4096ra1025nopf 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 4' || exit 1
echo done
