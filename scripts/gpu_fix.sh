# verification of the restored walk kernel + decision plane for narrow DPs only:
# SW/backtrace/chain GPU tests, then configs[2] / configs[3] / configs[1] GPU legs
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r02p; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sw.py tests/test_gpu_bt.py tests/test_gpu_chain.py tests/test_gpu_concurrency.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo tests ok
for m in ee paired local; do
  timeout -k 10 700 python -u bench.py --mode $m --no-cpu-baseline --server-sample 0 > $O/$m.json 2> $O/$m.log
  python3 -c "import json; d=json.loads(open('$O/$m.json').read().strip().splitlines()[-1]); print('$m', round(d['value']), round(d['ms_per_step'],1), {k: round(v,2) for k,v in d['kernels_ms'].items()})"
done
