#!/bin/bash
# r03q: the binding now sets 16 HW queues itself: drop-in at 3.1 Gbp with 2048 / 4096 / 8192
# workers (stock on the same box), DP dispatchers 2 vs 4; configs[0] with kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03q
mkdir -p $O
BT2G_ADAPTER_PROF=1 timeout -k 10 600 python -u scripts/longreads_bench.py --workers 512 > $O/longreads.json 2> $O/longreads.log || { tail $O/longreads.log; exit 1; }
mkdir -p /tmp/db3100
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 60 > $O/prof_$tag.txt
}
run g4096 4096 --reads 400000 --warmup-chunks 12 || exit 1
run g2048 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
BT2G_SEAM_THREADS_sw_dp=4 run g4096d4 4096 --reads 400000 --warmup-chunks 12 --skip-stock || exit 1
run g8192 8192 --reads 500000 --warmup-chunks 16 --skip-stock || exit 1
echo done
