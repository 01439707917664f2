# A/B: this tree's library vs exp/libbt2g_prev.so (the previous commit's):
# SW/backtrace/chain GPU tests, then the fill + backtrace bench (1M DPs) with
# alignments and edits compared
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sw.py tests/test_gpu_bt.py tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo tests ok
run() { echo "== $1"; env $2 timeout -k 10 200 python -u scripts/bt_bench.py --iters 3 $3 2>&1 | grep -E "lib=|compare"; }
run prev "BT2G_LIB=bowtie2-server_amd/exp/libbt2g_prev.so" "--save $O/p.npz"
run new "X=1" "--compare $O/p.npz"
rm -f $O/p.npz
