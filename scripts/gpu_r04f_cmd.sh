# round-4 GPU step: the GPU test suite and smoke() on the final tree
set -o pipefail
bash scripts/gpu_r04.sh tests r04ai
