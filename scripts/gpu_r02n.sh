set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02n
O=gpurun_out/r02n
timeout -k 10 400 python -u -m pytest tests/test_gpu_bt.py tests/test_gpu_sw.py tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests_sw.log 2>&1
echo tests ok
BT2G_BT_HPLANE=1 timeout -k 10 200 python -u scripts/bt_bench.py --save $O/ab_h.npz > $O/bt_h.log 2>&1
echo bt_h ok
timeout -k 10 200 python -u scripts/bt_bench.py --compare $O/ab_h.npz > $O/bt_dec.log 2>&1
echo bt_dec ok
rm -f $O/ab_h.npz
