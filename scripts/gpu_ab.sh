# A/B timing of fill + backtrace builds (scripts/bt_bench.py, 1M DPs); each
# line: label, env, library
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/ab; mkdir -p $O
run() { echo "== $1"; env $2 timeout -k 10 200 python -u scripts/bt_bench.py --iters 3 $3 2>&1 | grep -E "lib=|compare"; }
run h "BT2G_BT_HPLANE=1" "--save $O/h.npz"
run dec "X=1" "--compare $O/h.npz"
rm -f $O/h.npz
