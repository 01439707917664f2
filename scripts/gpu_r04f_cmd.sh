# round-4 GPU step: backtrace kernel tests, then batch-server runs (32 client connections, 8 warmup chunks)
set -o pipefail
mkdir -p gpurun_out/r04j
timeout -k 10 600 python -u -m pytest tests/test_gpu_bt.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04j/bt_tests.log 2>&1 || { tail -40 gpurun_out/r04j/bt_tests.log; exit 1; }
tail -3 gpurun_out/r04j/bt_tests.log
K=32 WARM=8 READS=400000 BT2G_KPROF=1 bash scripts/gpu_r04.sh batch r04j "16" && SKIP=--skip-stock K=32 WARM=8 READS=400000 bash scripts/gpu_r04.sh batch r04j "12"
