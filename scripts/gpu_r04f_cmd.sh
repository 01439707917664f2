# round-4 GPU step: the whole GPU test suite and smoke(), as the driver runs them
set -o pipefail
bash scripts/gpu_r04.sh tests r04ac
