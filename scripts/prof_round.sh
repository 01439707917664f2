# Full bench + rocprofv3 kernel stats of the same command (profiles/ evidence).
# Usage (on the GPU box): bash scripts/prof_round.sh <tag>
set -e
tag=${1:-r01}
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u bench.py --index-cache /tmp/bench_idx > gpurun_out/${tag}_bench.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- python3 bench.py --no-cpu-baseline --index-cache /tmp/bench_idx > gpurun_out/${tag}_prof.log 2>&1
