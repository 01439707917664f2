#!/bin/bash
# r03o: paired-step phase timing (the r02 paired regression); drop-in at
# 3.1 Gbp without the DP prefetch: per-kernel times of the seams' calls, more dispatchers for
# the saturated one_mm / DP seams, 4096 workers
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03o
mkdir -p $O
BT2G_BENCH_TIMING=1 timeout -k 10 900 python -u bench.py --mode paired --steps 2 --warmup 1 --no-cpu-baseline \
  > $O/paired.json 2> $O/paired.log || { tail -20 $O/paired.log; exit 1; }
mkdir -p /tmp/db3100 && for f in /tmp/bt2g_bench_index/hg38like_3100mb/g.*; do ln -sf $f /tmp/db3100/; done
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 60 > $O/prof_$tag.txt
}
BT2G_ADAPTER_PROF=1 run g2048k 2048 --reads 300000 --warmup-chunks 8 || exit 1
BT2G_SEAM_THREADS_one_mm=2 BT2G_SEAM_THREADS_sw_dp=4 run g2048d 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
BT2G_SEAM_THREADS_one_mm=2 BT2G_SEAM_THREADS_sw_dp=4 run g4096d 4096 --reads 400000 --warmup-chunks 12 --skip-stock || exit 1
echo done
