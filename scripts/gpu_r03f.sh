#!/bin/bash
# r03f: stock vs fiber drop-in on the 3.1 Gbp hg38-like genome (200 k reads)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03f
mkdir -p $O
BT2G_SAMPLE=$PWD/$O/samp_f2048.txt timeout -k 10 1100 python -u scripts/dropin_bench.py --genome-mb 3100 \
    --k 8 --gpu-workers 2048 --workdir /tmp/db3100 --reads 200000 --warmup-chunks 2 > $O/f2048.json 2> $O/f2048.log || exit 1
python scripts/prof_symbolize.py $O/samp_f2048.txt --top 60 > $O/prof_f2048.txt
echo done
