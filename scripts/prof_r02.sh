# Round-2 evidence: GPU tests, kernel-trace stats, separate FETCH_SIZE / WRITE_SIZE
# passes, then the bench line with roofline.traffic from those passes.
# Usage (on the GPU box): bash scripts/prof_r02.sh [tag]
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/${1:-r02}
mkdir -p $O
B="bench.py --no-cpu-baseline --index-cache /tmp/bench_idx"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
echo tests ok
timeout -k 10 500 python -u $B --steps 1 --warmup 0 > $O/idx.log 2>&1
echo index ok
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $B --steps 1 --warmup 0 > $O/pmc_fetch.log 2>&1
echo fetch ok
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $B --steps 1 --warmup 0 > $O/pmc_write.log 2>&1
echo write ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $B > $O/prof.log 2>&1
echo stats ok
timeout -k 10 600 python -u bench.py --index-cache /tmp/bench_idx --pmc-fetch $O/pmc_fetch/run_counter_collection.csv --pmc-write $O/pmc_write/run_counter_collection.csv > $O/bench.json 2> $O/bench.log
echo bench ok
