set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 600 python -u -m pytest tests/test_gpu_bt.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04f/bt_tests.log 2>&1 || { tail -30 gpurun_out/r04f/bt_tests.log; exit 1; }
tail -3 gpurun_out/r04f/bt_tests.log
BT2G_BATCH_SLOTS=4096 bash scripts/gpu_r04.sh batch r04f "16 8"
