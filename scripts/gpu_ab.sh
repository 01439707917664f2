# A/B timing of fill + backtrace variants (scripts/bt_bench.py, 1M DPs), all
# compared with the first run's alignments and edits
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/ab; mkdir -p $O
run() { echo "== $1"; env $2 timeout -k 10 200 python -u scripts/bt_bench.py --iters 3 $3 2>&1 | grep -E "lib=|compare|bt_"; }
run h_static "BT2G_BT_HPLANE=1 BT2G_BT_STATIC=1" "--save $O/h.npz"
run dec_static "BT2G_BT_STATIC=1" "--compare $O/h.npz"
run dec_queue "X=1" "--compare $O/h.npz"
run h_queue "BT2G_BT_HPLANE=1" "--compare $O/h.npz"
rm -f $O/h.npz
