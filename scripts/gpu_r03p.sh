#!/bin/bash
# r03p: the box's HW-queue setting and the fixed cost of one engine call (1 and 8 threads, 4 vs 16
# HW queues); configs[0] (longreads.fq) through the drop-in with 512 fibers; drop-in at 3.1 Gbp
# with 16 HW queues forced, kernel times on
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03p
mkdir -p $O
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset} nproc=$(nproc)" > $O/env.txt
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q BT2G_SYNC=poll timeout -k 10 300 python -u scripts/call_overhead.py --threads 1,8 --calls 100 \
    > $O/overhead_q$q.txt 2>&1 || { tail $O/overhead_q$q.txt; exit 1; }
done
timeout -k 10 600 python -u scripts/longreads_bench.py --workers 512 > $O/longreads.json 2> $O/longreads.log || { tail $O/longreads.log; exit 1; }
mkdir -p /tmp/db3100
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 60 > $O/prof_$tag.txt
}
GPU_MAX_HW_QUEUES=16 BT2G_ADAPTER_PROF=1 run g2048q16 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
echo done
