# round-4 GPU step: pinned-memory bandwidth, backtrace tests, batch server, bench
set -o pipefail
O=gpurun_out/r04y; mkdir -p $O
timeout -k 10 60 /opt/rocm/bin/hipcc -O2 --offload-arch=gfx950 scripts/micro/pinned_bw.cpp -o /tmp/pinned_bw && timeout -k 10 60 /tmp/pinned_bw > $O/pinned_bw.txt 2>&1; cat $O/pinned_bw.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_bt.py -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -le 1 ] || exit 1
K=32 WARM=8 READS=400000 BT2G_KPROF=1 bash scripts/gpu_r04.sh batch r04y "16" || exit 1
bash scripts/gpu_r04.sh bench r04y
