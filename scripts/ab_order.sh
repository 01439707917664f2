# A/B of the backtrace lane order (BT2G_BT_ORDER=0: problem order) on the three bench modes,
# then the GPU backtrace tests.  Usage (GPU box): bash scripts/ab_order.sh
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bt.py tests/test_gpu_sw.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests ok
B="bench.py --genome-mb 300 --index-cache /tmp/ab_idx --no-cpu-baseline --steps 3"
for m in ee local paired; do
  BT2G_BT_ORDER=0 timeout -k 10 300 python -u $B --mode $m > $O/${m}_0.log 2>&1
  echo $m 0 ok
  BT2G_BT_ORDER=1 timeout -k 10 300 python -u $B --mode $m > $O/${m}_1.log 2>&1
  echo $m 1 ok
done
