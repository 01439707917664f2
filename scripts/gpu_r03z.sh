#!/bin/bash
# r03z: the prefetched 1-mm search handed from the sweep's dispatcher to the 1-mm seam's queue
# (pipelined) -- drop-in SAM tests with the prefetch verified; prefetch on / off, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03z
mkdir -p $O /tmp/db3100
BT2G_SEEDPF_VERIFY=1 timeout -k 10 900 python -u -m pytest tests/test_integration.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 900 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers $w --workdir /tmp/db3100 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --role 1 --top 40 > $O/prof_$tag.txt
}
run g4096 4096 --reads 400000 --warmup-chunks 12 --dropin-args='--reads-per-batch 4' || exit 1
BT2G_SEEDPF=0 run g4096nopf 4096 --reads 400000 --warmup-chunks 12 --skip-stock --dropin-args='--reads-per-batch 4' || exit 1
echo done
