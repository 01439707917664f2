set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc$i -o run -- python3 scripts/bt_bench.py --iters 1 > gpurun_out/pmc$i.log 2>&1
done
