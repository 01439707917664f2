# r02n: GPU tests (all), then the default bench without the CPU legs
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
echo tests ok
timeout -k 10 600 python -u bench.py --no-cpu-baseline --server-sample 0 > $O/bench.json 2> $O/bench.log
echo bench ok
