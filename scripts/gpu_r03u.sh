#!/bin/bash
# r03u: decision plane for i16 end-to-end fills too (long reads: minsc < -254); SW / backtrace
# GPU tests, the drop-in SAM tests, configs[0] timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_sw.py tests/test_gpu_bt.py tests/test_gpu_chain.py tests/test_integration.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests failed; tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
BT2G_ADAPTER_PROF=1 timeout -k 10 600 python -u scripts/longreads_bench.py --workers 512 > $O/longreads.json 2> $O/longreads.log || { tail $O/longreads.log; exit 1; }
BT2G_ADAPTER_PROF=1 timeout -k 10 600 python -u scripts/longreads_bench.py --workers 2048 > $O/longreads2048.json 2> $O/longreads2048.log || { tail $O/longreads2048.log; exit 1; }
echo done
