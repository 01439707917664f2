#!/bin/bash
# r03w: decision plane for i16 end-to-end fills (long reads) + notify_all baton passed at unlock:
# SW / backtrace / chain GPU tests, drop-in SAM tests, configs[0] timing; drop-in read-ahead A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03w
mkdir -p $O /tmp/db3100
timeout -k 10 900 python -u -m pytest tests/test_gpu_sw.py tests/test_gpu_bt.py tests/test_gpu_chain.py tests/test_integration.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
BT2G_ADAPTER_PROF=1 timeout -k 10 600 python -u scripts/longreads_bench.py --workers 512 > $O/longreads.json 2> $O/longreads.log || { tail $O/longreads.log; exit 1; }
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_MUTEX_PROF=$PWD/$O/mx_$tag.txt BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 40 > $O/prof_$tag.txt
}
run g4096 4096 --reads 400000 --warmup-chunks 12 --dropin-args='--reads-per-batch 4' || exit 1
BT2G_READAHEAD=600 run g4096ra600 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 4' || exit 1
run g4096b2 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 2' || exit 1
echo done
