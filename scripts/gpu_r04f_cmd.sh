# round-4 GPU step: speculative DPs per ask and slots per driver, on one box
set -o pipefail
export K=32 WARM=8 READS=400000 SKIP=--skip-stock
bash scripts/gpu_r04.sh batch r04aa "16" || exit 1
BT2G_SPEC_DPS=8 bash scripts/gpu_r04.sh batch r04aa_spec8 "16" || exit 1
BT2G_SPEC_DPS=4 bash scripts/gpu_r04.sh batch r04aa_spec4 "16" || exit 1
BT2G_BATCH_SLOTS=1024 bash scripts/gpu_r04.sh batch r04aa_sl1k "16"
