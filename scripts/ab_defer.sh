# A/B: deferred gap tests in the end-to-end backtrace (libbt2g_defer.so, -DBT2G_BT_DEFER)
# vs the default build; GPU backtrace tests on both.  Usage (GPU box): bash scripts/ab_defer.sh
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/abdefer
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bt.py tests/test_gpu_sw.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests ok
BT2G_LIB=$PWD/bowtie2-server_amd/libbt2g_defer.so timeout -k 10 300 python -u -m pytest tests/test_gpu_bt.py -x -q --timeout 120 --timeout-method thread > $O/tests_defer.log 2>&1
echo tests defer ok
B="bench.py --genome-mb 300 --index-cache /tmp/ab_idx --steps 3 --cpu-sample 200000"
for m in ee paired; do
  timeout -k 10 300 python -u $B --mode $m > $O/${m}_base.log 2>&1
  echo $m base ok
  BT2G_LIB=$PWD/bowtie2-server_amd/libbt2g_defer.so timeout -k 10 300 python -u $B --mode $m > $O/${m}_defer.log 2>&1
  echo $m defer ok
done
