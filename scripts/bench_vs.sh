# BASELINE configs[4]'s per-GPU share: 10M / 8 = 1.25M 2 x 150 bp pairs, --very-sensitive,
# hg38-size genome, with the reference CPU baseline and parity.  Usage (GPU box): bash scripts/bench_vs.sh
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/vs
mkdir -p $O
timeout -k 10 900 python -u bench.py --mode paired --preset very-sensitive --reads 1250000 --cpu-sample 250000 > $O/bench.log 2>&1
echo bench ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke ok
