#!/bin/bash
# QLoRA decode prefetch: bitwise test, then Mistral-7B QLoRA on / off and the Mistral-7B-v0.3 bf16 LoRA in
# the same call (interleaved, two rounds)
set -o pipefail
mkdir -p gpurun_out/qlora_pf
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "qlora or nf4" > gpurun_out/qlora_pf/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/qlora_pf/pytest.log; [ $rc -eq 0 ] || exit $rc
OUT=qlora_pf ROUNDS=2 STEPS=6 WARMUP=2 STEP_TIMEOUT=400 BENCH_ARGS="--model mistral-7b --method qlora" ARMS="pf=FTC_NF4_PREFETCH=1 inline=FTC_NF4_PREFETCH=0" bash tools/step_ab.sh || exit 1
OUT=qlora_pf ROUNDS=1 STEPS=6 WARMUP=2 BENCH_ARGS="--model mistral-7b-v0.3" ARMS="lora_bf16=FTC_NF4_PREFETCH=1" bash tools/step_ab.sh
