#!/bin/bash
# Does hipBLASLt/rocBLAS offer faster solutions than the default heuristic for the LoRA step's GEMM
# shapes?  Same process layout as tools/pmc_gemms.py: default timing, then PyTorch TunableOp tuning
# (every candidate timed), then a run that only reads the tuned table.  -> gpurun_out/tunableop_probe/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
D=gpurun_out/tunableop_probe
mkdir -p $D
timeout -k 10 300 python tools/pmc_gemms.py --iters 20 --labels $D/labels.json > $D/default.log 2>&1 || exit 1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$D/tuned%d.csv \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-30} PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=0 \
  timeout -k 10 900 python tools/pmc_gemms.py --iters 3 --labels $D/labels.json > $D/tuning.log 2>&1 || exit 1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$D/tuned%d.csv \
  timeout -k 10 300 python tools/pmc_gemms.py --iters 20 --labels $D/labels.json > $D/tuned.log 2>&1 || exit 1
timeout -k 10 300 python tools/pmc_gemms.py --iters 20 --labels $D/labels.json > $D/default2.log 2>&1 || exit 1
paste <(grep '^{' $D/default.log | cut -c1-90) <(grep '^{' $D/tuned.log | sed 's/.*"ms"/"ms"/') <(grep '^{' $D/default2.log | sed 's/.*"ms"/"ms"/')
