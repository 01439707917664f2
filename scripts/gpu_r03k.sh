#!/bin/bash
# r03k: call overhead with one HW queue per stream; drop-in at 3.1 Gbp with fibers yielding on
# contended mutexes, read-ahead nthreads+1 per connection (A/B vs the reference's 4n+1), queue /
# resume delays per seam; carrier outboxes flushed during rounds (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03k
mkdir -p $O
GPU_MAX_HW_QUEUES=24 BT2G_SYNC=poll timeout -k 10 300 python -u scripts/call_overhead.py --threads 1,8 --calls 100 > $O/overhead_poll_q24.txt 2>&1 || exit 1
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 60 > $O/prof_$tag.txt
  for f in mprotect __lll_lock_wait_private __default_morecore malloc; do
    python scripts/prof_symbolize.py $O/samp_$tag.txt --callers-of $f --top 12 >> $O/callers_$tag.txt; done
}
BT2G_SEAM_THREADS=1 run g2048 2048 --reads 300000 --warmup-chunks 8 || exit 1
BT2G_SEAM_THREADS=1 BT2G_READAHEAD=999999 run g2048ra 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
BT2G_SEAM_THREADS=1 BT2G_FLUSH_US=10000000 BT2G_FLUSH_N=100000 run g2048f0 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
echo done
