# round-4 GPU step: GPU test suite + smoke with the wide decision plane defaults, then bench.py
set -o pipefail
bash scripts/gpu_r04.sh tests r04ae || exit 1
bash scripts/gpu_r04.sh bench r04ae
