#!/bin/bash
# Round-3 evidence, in gpurun calls of < 20 minutes each:
#   bash scripts/prof_r03.sh tests TAG   the whole GPU test suite, smoke()
#   bash scripts/prof_r03.sh prof  TAG   FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3 --pmc
#                                        runs of one bench step), kernel-trace stats of the bench
#   bash scripts/prof_r03.sh bench TAG   the bench line (roofline.traffic from the PMC CSVs of the
#                                        prof call, copied to profiles/r03/TAG/ in between), incl.
#                                        the CPU baseline and the real-schedule servers
#   bash scripts/prof_r03.sh modes TAG   --mode paired and --mode local lines with CPU baselines
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${2:-r03final}
P=profiles/r03/${2:-r03final}
mkdir -p $O
B="bench.py --no-cpu-baseline --server-sample 0"
pick() { find "$1" -name "*$2" | head -1; }
case "$1" in
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  echo smoke ok ;;
prof)
  timeout -s KILL 420 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $B --steps 1 --warmup 0 > $O/pmc_fetch.log 2>&1 || exit 1
  cp "$(pick $O/pmc_fetch counter_collection.csv)" $O/pmc_fetch.csv && echo fetch ok
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $B --steps 1 --warmup 0 > $O/pmc_write.log 2>&1 || exit 1
  cp "$(pick $O/pmc_write counter_collection.csv)" $O/pmc_write.csv && echo write ok
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $B > $O/prof.log 2>&1 || exit 1
  cp "$(pick $O/prof kernel_stats.csv)" $O/kernel_stats.csv && echo stats ok
  rm -rf $O/pmc_fetch $O/pmc_write $O/prof ;;
bench)
  timeout -k 10 1000 python -u bench.py --pmc-fetch $P/pmc_fetch.csv --pmc-write $P/pmc_write.csv > $O/bench.json 2> $O/bench.log || { tail -20 $O/bench.log; exit 1; }
  echo bench ok ;;
modes)
  timeout -k 10 540 python -u bench.py --mode paired --cpu-sample 200000 --server-sample 100000 > $O/paired_bench.json 2> $O/paired_bench.log || { tail $O/paired_bench.log; exit 1; }
  echo paired ok
  timeout -k 10 540 python -u bench.py --mode local --cpu-sample 200000 --server-sample 100000 > $O/local_bench.json 2> $O/local_bench.log || { tail $O/local_bench.log; exit 1; }
  echo local ok ;;
esac
