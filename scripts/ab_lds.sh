# A/B: backtrace tile valid bits in LDS (libbt2g.so) vs in the marks scratch (libbt2g_gv.so),
# after the GPU SW/backtrace tests.  Usage (GPU box): bash scripts/ab_lds.sh
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=gpurun_out/ablds
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bt.py tests/test_gpu_sw.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
echo tests ok
B="bench.py --genome-mb 300 --index-cache /tmp/ab_idx --no-cpu-baseline --steps 3"
for m in ee local paired; do
  BT2G_LIB=$PWD/bowtie2-server_amd/libbt2g_gv.so timeout -k 10 300 python -u $B --mode $m > $O/${m}_gv.log 2>&1
  echo $m gv ok
  timeout -k 10 300 python -u $B --mode $m > $O/${m}_lds.log 2>&1
  echo $m lds ok
done
