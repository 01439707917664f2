#!/bin/bash
# Round-4 GPU steps, one gpurun call each:
#   bash scripts/gpu_r04.sh gap TAG     kernel + HIP API trace of --mode paired (default path), gap summary
#   bash scripts/gpu_r04.sh tests TAG   the GPU test suite and smoke()
#   bash scripts/gpu_r04.sh batch TAG   the batch-first server vs the stock server (dropin_bench.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${2:-r04}
mkdir -p $O
# heartbeat: long index builds print nothing for minutes
( while sleep 50; do date +%T >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
case "$1" in
gap)
  timeout -k 10 600 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/ptrace -o run -- \
    python3 bench.py --mode paired --no-cpu-baseline --server-sample 0 --steps 2 --warmup 1 > $O/paired.json 2> $O/paired.log || { tail -20 $O/paired.log; exit 1; }
  python3 scripts/gap_trace.py $O/ptrace 15 > $O/gap.txt 2>&1; cat $O/gap.txt | head -80
  find $O/ptrace -name "*.csv" -size +20M -delete ;;
batch)
  # the batch-first server (integration/bt2g_batch.cpp) vs the stock server, configs[1] policy,
  # 3.1 Gbp hg38-like genome, 200 k reads, <= 10 k per connection, 8 connections
  for p in ${3:-32}; do
    BT2G_SAMPLE=$PWD/$O/samples_p$p.txt timeout -k 10 900 python3 -u scripts/dropin_bench.py --genome-mb 3100 --workdir /tmp/db \
      --dropin-binary integration/bin/bowtie2-align-server-batch --gpu-workers $p --k ${K:-8} --warmup-chunks ${WARM:-1} --reads ${READS:-200000} --mode ${MODE:-unpaired} ${SARGS:+--args=$SARGS} $SKIP > $O/batch_p$p.json 2> $O/batch_p$p.log \
      || { tail -30 $O/batch_p$p.log; tail -30 /tmp/db/server_dropin.log; exit 1; }
    cp /tmp/db/server_dropin.log $O/server_p$p.log
    SKIP=--skip-stock
    python3 -c "import json,sys; d=json.load(open('$O/batch_p$p.json')); print($p, {k: d[k] for k in ('sam_identical','speedup') if k in d}, d['dropin']['rate'], d['dropin']['server_cpu_s'], d['dropin'].get('engine_calls'))"
  done ;;
ktrace)
  # kernel trace of the batch server (rocprofv3 in front of the server's command line; the server
  # exits through exit() at SIGTERM so that the trace is written)
  p=${3:-16}
  timeout -k 10 900 python3 -u scripts/dropin_bench.py --genome-mb 3100 --reads ${4:-100000} --workdir /tmp/db \
    --dropin-binary integration/bin/bowtie2-align-server-batch --gpu-workers $p --skip-stock \
    --dropin-prefix "rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/ktrace -o run --" \
    > $O/ktrace_p$p.json 2> $O/ktrace_p$p.log || { tail -30 $O/ktrace_p$p.log; tail -30 /tmp/db/server_dropin.log; exit 1; }
  cp /tmp/db/server_dropin.log $O/server_ktrace.log
  python3 scripts/gap_trace.py $O/ktrace 10 > $O/ktrace_gap.txt 2>&1; head -60 $O/ktrace_gap.txt
  find $O/ktrace -name "*.csv" -size +40M -delete ;;
bench)
  # the driver's round-end command, as it runs it
  timeout -k 10 1100 python3 -u bench.py > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }
  cat $O/bench.json | cut -c1-1500 ;;
benchprof)
  # the same command with rocprofv3 --kernel-trace --stats in front of its batch server
  BT2G_BENCH_SERVER_PREFIX="rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/bprof -o run --" \
    timeout -k 10 1100 python3 -u bench.py --chain-steps 0 $BENCH_ARGS > $O/bench_prof.json 2> $O/bench_prof.log || { tail -30 $O/bench_prof.log; exit 1; }
  find $O/bprof -name "*kernel_stats.csv"
  find $O/bprof -name "*.csv" -size +40M -delete ;;
benchpmc)
  # separate FETCH_SIZE / WRITE_SIZE passes over the batch server's kernels (bench.py, 200 k reads)
  for c in FETCH_SIZE WRITE_SIZE; do
    BT2G_BENCH_SERVER_PREFIX="rocprofv3 --pmc $c --output-format csv -d $PWD/$O/pmc_$c -o run --" \
      timeout -k 10 900 python3 -u bench.py --chain-steps 0 --no-cpu-baseline --reads 200000 > $O/bench_pmc_$c.json 2> $O/bench_pmc_$c.log || { tail -30 $O/bench_pmc_$c.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/server_pmc.json
  find $O -name "*.csv" -size +40M -delete ;;
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  echo smoke ok ;;
esac
