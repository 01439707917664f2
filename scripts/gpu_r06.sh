#!/bin/bash
# Round-6 GPU steps, one gpurun call each:
#   bash scripts/gpu_r06.sh bench TAG          the driver's round-end command, as it runs it
#   bash scripts/gpu_r06.sh tests TAG          the GPU test suite and smoke()
#   bash scripts/gpu_r06.sh vs TAG             configs[4]'s per-GPU shard (paired --very-sensitive, 1.25 M pairs)
#   bash scripts/gpu_r06.sh prof TAG           rocprofv3 kernel trace of the bench command + FETCH/WRITE passes
#   bash scripts/gpu_r06.sh kprof TAG [STEPS]  the same kernel trace with the engines' HIP-event timing on (BT2G_KPROF)
#   bash scripts/gpu_r06.sh envab TAG [STEPS]  the bench under several server environments (ENVS="A=1;B=2"), REPS each
#   bash scripts/gpu_r06.sh mode TAG [STEPS]   another mode's line ($MODE local | paired, $PRESET) with a stock sample
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${2:-r06}
mkdir -p $O
( while sleep 50; do date +%T >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
summ() {  # one-line summary of a bench line
  python3 -c "
import json,sys; d=json.load(open('$1')); s=d['server']; k=d['server_kernels']
r=d.get('roofline') or {}
print('$2', round(d['value']), 'cpu_us', round(s['cpu_us_per_read'],1), 'busy', round(s['host_cores_busy'],1),
      'rss', s['server_rss_gb_per_pass'][-1], 'passes', [round(x,2) for x in s.get('pass_s',[])][:6],
      'fb', s.get('cpu_fallbacks'), 'roof', r.get('kernel','')[:30], r.get('frac'), 'vs', d.get('vs_cpu_baseline'),
      'sam', (d.get('sam_parity') or {}).get('identical'))
for kk in ('exact_sweep','seed_search','get_offset','ungapped','sw_dp'):
    c=s['calls'].get(kk)
    if c: print('  call', kk, c[2], 'calls', round(c[3]/max(1,c[2]),3), 'ms/call', round(c[0]/max(1,c[2])), 'req/call')
for kk,v in k.items(): print('  k', kk, v['kernel'][:28], v['launches'], round(v['ms_per_launch'],3), v.get('frac'))
"; }
case "$1" in
bench)
  T0=$(date +%s); timeout -k 10 1100 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }; echo "wall $(( $(date +%s) - T0 )) s"
  grep -v "^\s*$" $O/bench.log | tail -30; summ $O/bench.json bench ;;
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  echo smoke ok ;;
vs)
  T0=$(date +%s); timeout -k 10 1100 python3 -u bench.py --gpus 1 --mode paired --preset very-sensitive --reads 1250000 \
    --steps ${3:-2} --warmup 1 --chain-steps 0 > $O/bench_vs.json 2> $O/bench_vs.log || { tail -30 $O/bench_vs.log; exit 1; }
  echo "wall $(( $(date +%s) - T0 )) s"; summ $O/bench_vs.json vs ;;
mode)
  timeout -k 10 900 python3 -u bench.py --mode ${MODE:-local} --preset ${PRESET:-sensitive} --steps ${3:-1} --warmup 1 \
    --chain-steps 0 $BENCH_ARGS > $O/bench_${MODE:-local}.json 2> $O/bench_${MODE:-local}.log || { tail -30 $O/bench_${MODE:-local}.log; exit 1; }
  summ $O/bench_${MODE:-local}.json ${MODE:-local} ;;
prof)
  BT2G_BENCH_SERVER_PREFIX="rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/bprof -o run --" \
    timeout -k 10 600 python3 -u bench.py --steps 1 --warmup 1 --chain-steps 0 --stock-sample 0 --allow-fallbacks \
    > $O/bench_prof.json 2> $O/bench_prof.log || { tail -30 $O/bench_prof.log; exit 1; }
  find $O/bprof -name "*kernel_stats.csv" -exec cp {} $O/run_kernel_stats.csv \;
  find $O/bprof -name "*.csv" -size +40M -delete
  for c in FETCH_SIZE WRITE_SIZE; do
    BT2G_BENCH_SERVER_PREFIX="rocprofv3 --pmc $c --output-format csv -d $PWD/$O/pmc_$c -o run --" \
      timeout -k 10 500 python3 -u bench.py --steps 1 --warmup 1 --chain-steps 0 --stock-sample 0 --reads 200000 \
      --allow-fallbacks > $O/bench_pmc_$c.json 2> $O/bench_pmc_$c.log || { tail -30 $O/bench_pmc_$c.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/server_pmc.json $O/bench_pmc_FETCH_SIZE.json $O/bench_pmc_WRITE_SIZE.json
  find $O -name "*.csv" -size +40M -delete
  head -25 $O/run_kernel_stats.csv | cut -d, -f1-6 ;;
kprof)
  # rocprofv3 kernel trace of the bench command with the engines' own HIP-event timing on too
  # (BT2G_KPROF: the r04ag / r05h SIGSEGV under the profiler; events now made at context open)
  BT2G_BENCH_KPROF=1 BT2G_BENCH_SERVER_PREFIX="rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/kprof -o run --" \
    timeout -k 10 600 python3 -u bench.py --steps ${3:-2} --warmup 1 --chain-steps 0 --stock-sample 0 \
    > $O/bench_kprof.json 2> $O/bench_kprof.log || { tail -30 $O/bench_kprof.log; exit 1; }
  find $O/kprof -name "*kernel_stats.csv" -exec cp {} $O/kprof_kernel_stats.csv \;
  find $O/kprof -name "*.csv" -size +40M -delete
  summ $O/bench_kprof.json kprof; head -12 $O/kprof_kernel_stats.csv | cut -d, -f1-6 ;;
trace)
  # kernel + memory-copy trace of one pass (timeline of the calls: gaps between a stream's kernels and copies)
  BT2G_BENCH_SERVER_PREFIX="rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $PWD/$O/tprof -o run --" \
    timeout -k 10 600 python3 -u bench.py --steps 1 --warmup 1 --reads ${READS:-300000} --chain-steps 0 --stock-sample 0 --allow-fallbacks \
    > $O/bench_trace.json 2> $O/bench_trace.log || { tail -30 $O/bench_trace.log; exit 1; }
  find $O/tprof -name "*kernel_stats.csv" -exec cp {} $O/trace_kernel_stats.csv \;
  find $O/tprof -name "*memory_copy_stats.csv" -exec cp {} $O/trace_copy_stats.csv \;
  python3 scripts/trace_gaps.py $O/tprof > $O/trace_gaps.txt 2>&1; tail -40 $O/trace_gaps.txt
  find $O/tprof -name "*.csv" -size +60M -delete ;;
cpuprof)
  # the batch server's per-read logic by phase ($BT2G_PHASES) and a flat CPU profile of its threads ($BT2G_SAMPLE)
  BT2G_PHASES=1 BT2G_SAMPLE=$PWD/$O/samples.txt timeout -k 10 600 python3 -u bench.py --steps ${3:-3} --warmup 1 --chain-steps 0 \
    --stock-sample 0 $BENCH_ARGS > $O/bench_phases.json 2> $O/bench_phases.log || { tail -30 $O/bench_phases.log; exit 1; }
  cp integration/bin/bowtie2-align-server-batch $O/server.bin
  summ $O/bench_phases.json phases ;;
fmtests)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_fm.py tests/test_batch.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/fm_tests.log 2>&1 || { tail -20 $O/fm_tests.log; exit 1; }
  tail -2 $O/fm_tests.log ;;
diag)
  bash $0 tests $2 && bash $0 quick $2 && bash $0 trace $2 ;;
quick)
  timeout -k 10 700 python3 -u bench.py --gpus 1 --steps ${3:-3} --warmup 1 --chain-steps 0 > $O/bench_quick.json 2> $O/bench_quick.log || { tail -30 $O/bench_quick.log; exit 1; }
  summ $O/bench_quick.json quick ;;
envab)
  # bench.py under several server environments: ENVS="A=1 B=2;A=3" (';' between settings), REPS rounds, interleaved
  IFS=';' read -ra SETS <<< "${ENVS:-BT2G_DP_WORKERS=6}"
  for rep in $(seq 1 ${REPS:-1}); do
    i=0
    for set in "${SETS[@]}"; do
      i=$((i+1))
      env $set timeout -k 10 500 python3 -u bench.py --mode ${MODE:-ee} --steps ${3:-2} --warmup 1 --chain-steps 0 --stock-sample 0 $BENCH_ARGS \
        > $O/bench_${i}_$rep.json 2> $O/bench_${i}_$rep.log || { tail -30 $O/bench_${i}_$rep.log; exit 1; }
      summ $O/bench_${i}_$rep.json "[$set] rep $rep"
    done
  done ;;
esac
