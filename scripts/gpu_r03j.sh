#!/bin/bash
# r03j: engine call overhead microbench; RCCL counter all-reduce + two-replica drop-in tests;
# drop-in at 3.1 Gbp with one dispatcher per seam and 4096 / 8192 workers
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 300 python -u scripts/call_overhead.py --threads 1,4,8 --calls 100 > $O/overhead_spin.txt 2>&1 || exit 1
BT2G_SYNC=poll timeout -k 10 300 python -u scripts/call_overhead.py --threads 1,4,8 --calls 100 > $O/overhead_poll.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_fm.py tests/test_integration.py -m gpu -k "comm or two_replicas or brq or golden" \
  -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 60 > $O/prof_$tag.txt
}
BT2G_SEAM_THREADS=1 run g4096s1 4096 --reads 400000 --warmup-chunks 12 --skip-stock || exit 1
BT2G_SEAM_THREADS=1 run g8192s1 8192 --reads 400000 --warmup-chunks 16 --skip-stock || exit 1
echo done
