# configs[2] (paired) and configs[3] (local) on the 3.1 Gbp hg38-like genome,
# GPU legs only (the index is built once and cached under $TMPDIR)
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r02o; mkdir -p $O
timeout -k 10 700 python -u bench.py --mode paired --no-cpu-baseline --server-sample 0 > $O/paired.json 2> $O/paired.log
echo paired ok
timeout -k 10 500 python -u bench.py --mode local --no-cpu-baseline --server-sample 0 > $O/local.json 2> $O/local.log
echo local ok
