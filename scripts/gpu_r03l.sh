#!/bin/bash
# r03l: packed DP outputs written straight to pinned memory (one sync per DP call), one dispatcher
# per seam by default; SAM parity; drop-in at 3.1 Gbp with 2048 / 3072 / 4096 workers
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_bt.py tests/test_gpu_concurrency.py tests/test_integration.py -m gpu \
  -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 60 > $O/prof_$tag.txt
}
run g2048 2048 --reads 300000 --warmup-chunks 8 || exit 1
run g3072 3072 --reads 300000 --warmup-chunks 10 --skip-stock || exit 1
run g4096 4096 --reads 400000 --warmup-chunks 12 --skip-stock || exit 1
echo done
