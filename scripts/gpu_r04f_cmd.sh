# round-4 GPU step: batch-server runs (p 16 / 8) then a kernel trace at p 16
set -o pipefail
bash scripts/gpu_r04.sh batch r04g "16 8" && bash scripts/gpu_r04.sh ktrace r04g 16 100000
