#!/bin/bash
# r03a: the drop-in server with fiber workers vs the stock server (200 Mbp
# hg38-like genome, 200 k reads), plus OS-thread workers and a CPU profile.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03a
mkdir -p $O
export BT2G_SAMPLE=$PWD/$O/samp_f1024.txt
timeout -k 10 600 python -u scripts/dropin_bench.py --genome-mb 200 --reads 200000 --k 8 --gpu-workers 1024 \
  --workdir /tmp/db200 > $O/f1024.json 2> $O/f1024.log || exit 1
python scripts/prof_symbolize.py $BT2G_SAMPLE --top 90 > $O/prof_f1024.txt
export BT2G_SAMPLE=$PWD/$O/samp_f2048.txt
timeout -k 10 400 python -u scripts/dropin_bench.py --genome-mb 200 --reads 200000 --k 8 --gpu-workers 2048 \
  --workdir /tmp/db200 --skip-stock > $O/f2048.json 2> $O/f2048.log || exit 1
python scripts/prof_symbolize.py $BT2G_SAMPLE --top 90 > $O/prof_f2048.txt
unset BT2G_SAMPLE
BT2G_FIBERS=0 timeout -k 10 400 python -u scripts/dropin_bench.py --genome-mb 200 --reads 200000 --k 8 --gpu-workers 1024 \
  --workdir /tmp/db200 --skip-stock > $O/t1024.json 2> $O/t1024.log || exit 1
echo done
