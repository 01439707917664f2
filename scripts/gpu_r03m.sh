#!/bin/bash
# r03m: speculative DP prefetch, caching operator new, per-fiber driver tables; SAM parity;
# drop-in at 3.1 Gbp with A/Bs (prefetch off, glibc allocator, 2 one_mm dispatchers)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03m
mkdir -p $O
BT2G_SPEC_VERIFY=1 timeout -k 10 900 python -u -m pytest tests/test_integration.py -m gpu \
  -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 60 > $O/prof_$tag.txt
}
BT2G_SPEC_VERIFY=1 run g2048v 2048 --reads 100000 --warmup-chunks 4 || exit 1
run g2048 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
BT2G_SPEC=0 run g2048nospec 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
BT2G_ALLOC=0 run g2048glibc 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
BT2G_SEAM_THREADS_one_mm=2 BT2G_SEAM_THREADS_extend=2 run g2048mm2 2048 --reads 300000 --warmup-chunks 8 --skip-stock || exit 1
echo done
