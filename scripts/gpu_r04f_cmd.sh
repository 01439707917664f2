# round-4 GPU step: FM/backtrace tests, batch server p16 (seed call with its ranges' extension
# and rows), the same without (BT2G_SEED_PREFETCH=0), then the pinned variant
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fm.py tests/test_gpu_bt.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
{ cat /sys/fs/cgroup/cpu.max; cat /sys/fs/cgroup/cpu.stat; nproc; } > $O/cgroup_before.txt 2>&1
K=32 WARM=8 READS=400000 BT2G_KPROF=1 BT2G_ALLOC_XTRACE=1 BT2G_ALLOC_STATS=$PWD/$O/alloc_p16.txt \
  bash scripts/gpu_r04.sh batch r04p "16" || exit 1
cat /sys/fs/cgroup/cpu.stat > $O/cgroup_after.txt 2>&1
SKIP=--skip-stock K=32 WARM=8 READS=400000 BT2G_SEED_PREFETCH=0 bash scripts/gpu_r04.sh batch r04p_nosd "16" || exit 1
SKIP=--skip-stock K=32 WARM=8 READS=400000 BT2G_PIN_CPUS=auto bash scripts/gpu_r04.sh batch r04p_pin "16"
