#!/bin/bash
# BASELINE.json configs on one MI355X: ours (HIP kernels) and the stock PyTorch-ROCm path.
# Usage (GPU box): bash tools/bench_configs.sh [name ...]   (default: all)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/configs
declare -A CMD=(
  [lora]="--steps 10 --warmup 3"
  [lora_torch]="--steps 5 --warmup 2 --kernels torch"
  [qlora_mistral]="--model mistral-7b --method qlora --steps 5 --warmup 2"
  [qlora_mistral_torch]="--model mistral-7b --method qlora --steps 3 --warmup 2 --kernels torch"
  [full]="--method full --steps 5 --warmup 2"
  [full_torch]="--method full --steps 3 --warmup 2 --kernels torch"
  [llama32_1b]="--model llama3.2-1b --steps 10 --warmup 3"
  [llama32_3b]="--model llama3.2-3b --steps 10 --warmup 3"
  [mistral_lora]="--model mistral-7b-v0.3 --steps 8 --warmup 3"
  [long_16k]="--batch-size 2 --seq-len 16384 --steps 4 --warmup 2"
  [long_32k]="--batch-size 1 --seq-len 32768 --steps 4 --warmup 2"
  [packed_512]="--doc-len 512 --steps 8 --warmup 3"
  [full_fp32_accum2]="--method full --grad-accum 2 --grad-dtype fp32 --steps 3 --warmup 1"
)
NAMES=("$@")
[ ${#NAMES[@]} -eq 0 ] && NAMES=(lora qlora_mistral full lora_torch qlora_mistral_torch full_torch)
for n in "${NAMES[@]}"; do
  timeout -k 10 900 python bench.py ${CMD[$n]} > gpurun_out/configs/$n.log 2>&1
  rc=$?
  echo "[$n] rc=$rc $(tail -1 gpurun_out/configs/$n.log | cut -c1-400)"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping"; exit $rc; fi
done
