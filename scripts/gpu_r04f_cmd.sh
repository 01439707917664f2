# round-4 GPU step: bench.py as the driver runs it, then with rocprofv3 in front of its batch server
set -o pipefail
bash scripts/gpu_r04.sh bench r04t || exit 1
bash scripts/gpu_r04.sh benchprof r04t
