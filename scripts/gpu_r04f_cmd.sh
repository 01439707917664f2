# round-4 GPU step: backtrace tests, the backtrace kernels at a batch-server batch size, batch server p16
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_bt.py -x -v --timeout 300 --timeout-method thread > $O/bt_tests.log 2>&1 || { tail -40 $O/bt_tests.log; exit 1; }
tail -2 $O/bt_tests.log
for v in wg:8192:1 lds:8192:0 lane:0:1; do
  IFS=: read name lim wg <<< "$v"
  BT2G_BT_LDS_MAX=$lim BT2G_BT_WG=$wg timeout -k 10 300 python -u scripts/bt_bench.py --n 1600 --iters 5 > $O/btb_$name.log 2>&1 || { tail -20 $O/btb_$name.log; exit 1; }
  echo "== $name"; tail -3 $O/btb_$name.log
done
K=32 WARM=8 READS=400000 BT2G_KPROF=1 bash scripts/gpu_r04.sh batch r04k "16"
