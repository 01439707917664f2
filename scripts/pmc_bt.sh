# PMC passes over scripts/bt_bench.py (1M end-to-end DPs, fill + backtrace),
# one rocprofv3 --pmc run per counter group; BT2G_BT_HPLANE=1 in the
# environment profiles the H score plane instead of the decision plane.
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/pmc}
mkdir -p $O
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc$i -o run -- python3 scripts/bt_bench.py --iters 1 > $O/pmc$i.log 2>&1
  echo pass $i ok
done
