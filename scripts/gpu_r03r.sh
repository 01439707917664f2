#!/bin/bash
# r03r: smaller read batches per worker element for the drop-in (--reads-per-batch: a worker
# aligns its element's reads one after another, so a connection lasts >= batch x per-read
# latency), big blocks in the caching allocator, shorter mutex spins; contended-lock sites
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03r
mkdir -p $O /tmp/db3100
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_MUTEX_PROF=$PWD/$O/mx_$tag.txt BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 60 > $O/prof_$tag.txt
}
run g2048b4 2048 --reads 300000 --warmup-chunks 8 --dropin-args='--reads-per-batch 4' || exit 1
run g4096b4 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 4' || exit 1
run g4096b1 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 1' || exit 1
run g8192b2 8192 --reads 500000 --warmup-chunks 16 --skip-stock --dropin-args='--reads-per-batch 2' || exit 1
echo done
