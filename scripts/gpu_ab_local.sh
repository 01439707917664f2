# A/B of the local fill: this tree's library vs exp/libbt2g_prev.so (the
# previous commit's): SW and chain GPU tests, then --mode local benches on a
# 200 Mbp hg38-like genome (200 k reads)
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sw.py tests/test_gpu_bt.py tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_local.log 2>&1
echo tests ok
for L in prev new prev new; do
  if [ $L = prev ]; then export BT2G_LIB=bowtie2-server_amd/exp/libbt2g_prev.so; else unset BT2G_LIB; fi
  timeout -k 10 300 python -u bench.py --mode local --genome-mb 200 --reads 200000 --steps 3 --warmup 1 --no-cpu-baseline --server-sample 0 2> $O/local_$L.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L', round(d['value']), {k: round(v, 2) for k, v in d['kernels_ms'].items()})"
done
run() { echo "== $1"; env $2 timeout -k 10 200 python -u scripts/bt_bench.py --iters 3 $3 2>&1 | grep -E "lib=|compare"; }
run prev "BT2G_LIB=bowtie2-server_amd/exp/libbt2g_prev.so" "--save $O/p.npz"
run new "X=1" "--compare $O/p.npz"
rm -f $O/p.npz
