# A/B of backtrace builds (scripts/bt_bench.py, 1M DPs), alignments and edits
# compared with the first run's
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/ab; mkdir -p $O
run() { echo "== $1"; env $2 timeout -k 10 200 python -u scripts/bt_bench.py --iters 3 $3 2>&1 | grep -E "lib=|compare"; }
run base "X=1" "--save $O/p.npz"
run chunk6 "BT2G_LIB=bowtie2-server_amd/exp/libbt2g_chunk6.so" "--compare $O/p.npz"
run chunk8 "BT2G_LIB=bowtie2-server_amd/exp/libbt2g_chunk8.so" "--compare $O/p.npz"
rm -f $O/p.npz
