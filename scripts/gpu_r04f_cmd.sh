# round-4 GPU step: bench.py as the driver runs it
set -o pipefail
bash scripts/gpu_r04.sh bench r04s
