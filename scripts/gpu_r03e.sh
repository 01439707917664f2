#!/bin/bash
# r03e: poll-based stream waits in the dispatchers; sampler with thread roles
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03e
mkdir -p $O
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 500 python -u scripts/dropin_bench.py --genome-mb 200 \
    --k 8 --gpu-workers $w --workdir /tmp/db200 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --top 60 > $O/prof_$tag.txt
  python scripts/prof_symbolize.py $O/samp_$tag.txt --callers-of mprotect --top 10 > $O/mprotect_$tag.txt
  python scripts/prof_symbolize.py $O/samp_$tag.txt --callers-of nanosleep --top 10 > $O/sleep_$tag.txt
}
run f1024 1024 --reads 300000 --warmup-chunks 3 || exit 1
run f2048 2048 --reads 300000 --warmup-chunks 3 --skip-stock || exit 1
BT2G_CARRIERS=12 run f2048c12 2048 --reads 300000 --warmup-chunks 3 --skip-stock || exit 1
echo done
