#!/bin/bash
# TunableOp over the FULL fine-tuning step's GEMMs (forward, TN input-gradient and the weight-gradient
# shapes dW += dy^T x that the LoRA step never runs), then the bench reading the tuned table, and an
# untuned bench in the same call for the A/B.  -> gpurun_out/tune_full/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
D=gpurun_out/tune_full
mkdir -p $D
timeout -k 10 600 python bench.py --method full --steps 5 --warmup 2 > $D/bench_default.log 2>&1 || exit 1
grep '^{' $D/bench_default.log | cut -c1-200
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$D/tuned%d.csv \
  PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-30} PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=0 \
  PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 900 python bench.py --method full --steps 1 --warmup 1 > $D/tuning.log 2>&1 || exit 1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$D/tuned%d.csv \
  timeout -k 10 600 python bench.py --method full --steps 5 --warmup 2 > $D/bench_tuned.log 2>&1 || exit 1
grep '^{' $D/bench_tuned.log | cut -c1-200
timeout -k 10 600 python bench.py --method full --steps 5 --warmup 2 > $D/bench_default2.log 2>&1 || exit 1
grep '^{' $D/bench_default2.log | cut -c1-200
