#!/bin/bash
# r03i: cache slots reserved (no fill), one H2D / one D2H per engine call, one HIP
# hardware queue per stream; drop-in vs stock at 3.1 Gbp, A/B of the queue count
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fm.py tests/test_gpu_concurrency.py tests/test_gpu_sw.py -x -q \
  --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 60 > $O/prof_$tag.txt
}
run g2048 2048 --reads 300000 --warmup-chunks 8 || exit 1
GPU_MAX_HW_QUEUES=4 run g2048q4 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
BT2G_SEAM_THREADS=1 run g2048s1 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
echo done
