# VALU instructions of the SW fill per DP cell: one rocprofv3 --pmc pass over
# scripts/bt_bench.py (1M DPs of 150 x 210 cells) for the decision-plane fill
# and one for the H-plane fill (BT2G_BT_HPLANE=1)
set -e
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_fill; mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --output-format csv -d $O/dec -o run -- python3 scripts/bt_bench.py --iters 1 > $O/dec.log 2>&1
echo dec ok
BT2G_BT_HPLANE=1 timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU --output-format csv -d $O/h -o run -- python3 scripts/bt_bench.py --iters 1 > $O/h.log 2>&1
echo h ok
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke ok
