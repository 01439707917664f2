# A/B of the bench step: seeds concurrent with the 1-mm search (default) vs
# serial (BT2G_BENCH_SERIAL=1), 3.1 Gbp hg38-like genome; chain parity test first
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo tests ok
for v in serial conc; do
  if [ $v = serial ]; then export BT2G_BENCH_SERIAL=1; else unset BT2G_BENCH_SERIAL; fi
  timeout -k 10 600 python -u bench.py --no-cpu-baseline --server-sample 0 --steps 5 > $O/bench_$v.json 2> $O/bench_$v.log
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['kernels_ms'])"
done
