#!/bin/bash
# r03g: GPU tests after the driver seams (extend, SA rows) + drop-in A/B at 200 Mbp
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 500 python -u scripts/dropin_bench.py --genome-mb 200 \
    --k 8 --gpu-workers $w --workdir /tmp/db200 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --top 50 > $O/prof_$tag.txt
}
run f2048 2048 --reads 300000 --warmup-chunks 3 || exit 1
BT2G_SEAM_THREADS=1 run f2048s1 2048 --reads 300000 --warmup-chunks 3 --skip-stock || exit 1
BT2G_SEAM_THREADS=1 BT2G_BATCH_WINDOW_US=600 run f2048s1w600 2048 --reads 300000 --warmup-chunks 3 --skip-stock || exit 1
echo done
