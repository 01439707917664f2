#!/bin/bash
# r03c: fiber drop-in with a warm-up connection; callers of mprotect
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03c
mkdir -p $O
run() {   # tag workers extra-args...
  local tag=$1 w=$2; shift 2
  BT2G_SAMPLE=$PWD/$O/samp_$tag.txt timeout -k 10 400 python -u scripts/dropin_bench.py --genome-mb 200 --reads 200000 \
    --k 8 --gpu-workers $w --workdir /tmp/db200 "$@" > $O/$tag.json 2> $O/$tag.log || return 1
  python scripts/prof_symbolize.py $O/samp_$tag.txt --top 70 > $O/prof_$tag.txt
  python scripts/prof_symbolize.py $O/samp_$tag.txt --callers-of mprotect --top 20 > $O/mprotect_$tag.txt
  python scripts/prof_symbolize.py $O/samp_$tag.txt --callers-of hsa_amd_image --top 20 > $O/hsa_$tag.txt
}
run f1024 1024 || exit 1
run f4096 4096 --skip-stock || exit 1
run f2048 2048 --skip-stock || exit 1
echo done
