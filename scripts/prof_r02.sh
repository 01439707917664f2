# Round-2 evidence, in two gpurun calls (each under the 20-minute limit):
#   bash scripts/prof_r02.sh prof  TAG   GPU tests, FETCH_SIZE and WRITE_SIZE passes (separate
#                                        rocprofv3 --pmc runs), kernel-trace stats
#   bash scripts/prof_r02.sh bench TAG   the bench line, roofline.traffic from the PMC CSVs of the
#                                        first call (copied to profiles/TAG/ in between)
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/${2:-r02}
mkdir -p $O
B="bench.py --no-cpu-baseline --server-sample 0"
if [ "$1" = prof ]; then
  timeout -k 10 720 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1
  echo tests ok
  timeout -s KILL 360 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $B --steps 1 --warmup 0 > $O/pmc_fetch.log 2>&1
  echo fetch ok
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $B --steps 1 --warmup 0 > $O/pmc_write.log 2>&1
  echo write ok
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $B > $O/prof.log 2>&1
  echo stats ok
else
  P=profiles/${2:-r02}
  timeout -k 10 900 python -u bench.py --pmc-fetch $P/pmc_fetch.csv --pmc-write $P/pmc_write.csv > $O/bench.json 2> $O/bench.log
  echo bench ok
fi
