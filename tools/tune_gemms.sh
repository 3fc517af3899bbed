#!/bin/bash
# Tune hipBLASLt/rocBLAS GEMM solutions for the flagship bench shapes with PyTorch TunableOp,
# then re-run the bench reading the tuned table.  Result table -> gpurun_out/tunableop/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/tunableop
export PYTORCH_TUNABLEOP_ENABLED=1
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop/tunableop_results%d.csv
export PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-20}
export PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=0
PYTORCH_TUNABLEOP_TUNING=1 timeout -k 10 ${TUNE_TIMEOUT:-900} python bench.py --steps 2 --warmup 1 \
  > gpurun_out/tunableop/tune.log 2>&1 || { echo "tuning rc=$?"; tail -5 gpurun_out/tunableop/tune.log; exit 1; }
tail -1 gpurun_out/tunableop/tune.log
PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 600 python bench.py --steps 10 --warmup 3 \
  > gpurun_out/tunableop/bench_tuned.log 2>&1 || { echo "tuned bench rc=$?"; exit 1; }
tail -1 gpurun_out/tunableop/bench_tuned.log
