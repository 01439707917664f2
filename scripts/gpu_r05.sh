#!/bin/bash
# Round-5 GPU steps, one gpurun call each:
#   bash scripts/gpu_r05.sh mem TAG [STEPS]   bench.py's batch server over STEPS passes: RSS per pass, THP mode
#   bash scripts/gpu_r05.sh bench TAG         the driver's round-end command, as it runs it
#   bash scripts/gpu_r05.sh tests TAG         the GPU test suite and smoke()
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${2:-r05}
mkdir -p $O
( while sleep 50; do date +%T >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
case "$1" in
mem)
  cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag > $O/thp.txt 2>&1
  free -g >> $O/thp.txt 2>&1; cat $O/thp.txt
  timeout -k 10 800 python3 -u bench.py --steps ${3:-6} --warmup 1 --chain-steps 0 --stock-sample 0 $BENCH_ARGS \
    > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }
  grep "RSS\|real schedule" $O/bench.log
  python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['server'])[:3000])" ;;
slots)
  # the batch server at several slot caps (reads in flight per driver): rate, RSS, CPU per read
  for S in ${SLOTS:-1024 768}; do
    BT2G_BATCH_SLOTS=$S timeout -k 10 500 python3 -u bench.py --steps ${3:-3} --warmup 1 --chain-steps 0 --stock-sample 0 $BENCH_ARGS \
      > $O/bench_s$S.json 2> $O/bench_s$S.log || { tail -30 $O/bench_s$S.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_s$S.json')); s=d['server']; print($S, round(d['value']), s['slots'], s['server_rss_gb_per_pass'], round(s['cpu_us_per_read'],1))"
  done ;;
phases)
  # the batch server's per-read logic by phase ($BT2G_PHASES) and a flat CPU profile ($BT2G_SAMPLE)
  BT2G_PHASES=1 BT2G_SAMPLE=$PWD/$O/samples.txt timeout -k 10 600 python3 -u bench.py --steps ${3:-2} --warmup 1 --chain-steps 0 \
    --stock-sample 0 $BENCH_ARGS > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }
  cp integration/bin/bowtie2-align-server-batch $O/server.bin
  python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['server']['cpu_us_per_read'])" ;;
drivers)
  # driver threads x slots per driver: "D:S D:S ..." ($DS)
  for ds in ${DS:-24:683 20:820}; do
    D=${ds%%:*}; S=${ds##*:}
    BT2G_BATCH_SLOTS=$S timeout -k 10 500 python3 -u bench.py --drivers $D --steps ${3:-3} --warmup 1 --chain-steps 0 --stock-sample 0 $BENCH_ARGS \
      > $O/bench_d$D.json 2> $O/bench_d$D.log || { tail -30 $O/bench_d$D.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_d$D.json')); s=d['server']; print($D, $S, round(d['value']), s['slots'], s['server_rss_gb_per_pass'][-1], round(s['cpu_us_per_read'],1), s['idle_ms'])"
  done ;;
prof)
  # rocprofv3 kernel trace of the bench command's batch server (default path: the workgroup
  # walk with its LDS opt-in), then the FETCH_SIZE / WRITE_SIZE passes (separate runs)
  BT2G_BENCH_SERVER_PREFIX="rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/$O/bprof -o run --" \
    timeout -k 10 600 python3 -u bench.py --steps 1 --warmup 1 --chain-steps 0 --stock-sample 0 > $O/bench_prof.json 2> $O/bench_prof.log || { tail -30 $O/bench_prof.log; exit 1; }
  find $O/bprof -name "*kernel_stats.csv" -exec cp {} $O/run_kernel_stats.csv \;
  find $O/bprof -name "*.csv" -size +40M -delete
  for c in FETCH_SIZE WRITE_SIZE; do
    BT2G_BENCH_SERVER_PREFIX="rocprofv3 --pmc $c --output-format csv -d $PWD/$O/pmc_$c -o run --" \
      timeout -k 10 500 python3 -u bench.py --steps 1 --warmup 1 --chain-steps 0 --stock-sample 0 --reads 200000 > $O/bench_pmc_$c.json 2> $O/bench_pmc_$c.log || { tail -30 $O/bench_pmc_$c.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/server_pmc.json
  find $O -name "*.csv" -size +40M -delete
  head -25 $O/run_kernel_stats.csv | cut -d, -f1-6 ;;
mode)
  # one bench line of another mode ($MODE: local | paired; $PRESET) with the stock server on 200 k
  timeout -k 10 900 python3 -u bench.py --mode ${MODE:-local} --preset ${PRESET:-sensitive} --steps ${3:-1} --warmup 1 \
    --chain-steps 0 --stock-sample 200000 $BENCH_ARGS > $O/bench_${MODE:-local}.json 2> $O/bench_${MODE:-local}.log || { tail -30 $O/bench_${MODE:-local}.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_${MODE:-local}.json')); s=d['server']
print(round(d['value']), d['vs_cpu_baseline'], d['sam_parity'], s['cpu_us_per_read'], s['server_rss_gb_per_pass'])
for k, v in d['server_kernels'].items(): print(k, v['kernel'][:40], v['launches'], round(v['ms_per_launch'], 3), v.get('frac'))" ;;
localab)
  # the local walk variants through the batch server ($BT2G_BT_LOC_LDS: marks | plane | 0)
  timeout -k 10 300 python -u -m pytest tests/test_gpu_bt.py -x -q --timeout 200 --timeout-method thread > $O/bt_tests.log 2>&1 || { tail -30 $O/bt_tests.log; exit 1; }
  tail -1 $O/bt_tests.log
  for v in ${VARS:-marks plane}; do
    BT2G_BT_LOC_LDS=$v timeout -k 10 500 python3 -u bench.py --mode local --steps 1 --warmup 1 --chain-steps 0 --stock-sample 0 $BENCH_ARGS \
      > $O/bench_$v.json 2> $O/bench_$v.log || { tail -30 $O/bench_$v.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$v.json')); k=d['server_kernels']; print('$v', round(d['value']), round(k['sw_dp:5']['ms_per_launch'],2), round(k['sw_dp:7']['ms_per_launch'],2), round(k['exact_sweep:2']['ms_per_launch'],2))"
  done ;;
envab)
  # bench.py --mode $MODE under several server environments: ENVS="A=1 B=2;A=3" (';' between settings)
  IFS=';' read -ra SETS <<< "${ENVS:-BT2G_DP_WORKERS=6}"
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    env $set timeout -k 10 500 python3 -u bench.py --mode ${MODE:-local} --steps ${3:-1} --warmup 1 --chain-steps 0 --stock-sample 0 $BENCH_ARGS \
      > $O/bench_$i.json 2> $O/bench_$i.log || { tail -30 $O/bench_$i.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$i.json')); s=d['server']; k=d['server_kernels']; print('$set', round(d['value']), round(s['cpu_us_per_read'],1), s['server_rss_gb_per_pass'][-1], round(k['sw_dp:7']['ms_per_launch'],2), k['sw_dp:7']['launches'])"
  done ;;
clientab)
  # the timed passes with the multi-connection client and with the reference client
  for c in ${CLIENTS:-native reference}; do
    timeout -k 10 500 python3 -u bench.py --client $c --steps ${3:-3} --warmup 1 --chain-steps 0 --stock-sample 0 $BENCH_ARGS \
      > $O/bench_$c.json 2> $O/bench_$c.log || { tail -30 $O/bench_$c.log; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_$c.json')); s=d['server']; print('$c', round(d['value']), round(s['cpu_us_per_read'],1), round(s['client_cpu_us_per_read'],2), s['server_rss_gb_per_pass'][-1])"
  done ;;
bench)
  T0=$(date +%s); timeout -k 10 1100 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { tail -30 $O/bench.log; exit 1; }; echo "wall $(( $(date +%s) - T0 )) s"
  tail -25 $O/bench.log | grep -v "^\s*$"; cut -c1-1500 $O/bench.json ;;
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  echo smoke ok ;;
esac
