#!/bin/bash
# QLoRA decode prefetch A/B (Mistral-7B QLoRA, prefetch on / off) with the Mistral-7B-v0.3 bf16 LoRA control,
# interleaved, three rounds
set -o pipefail
mkdir -p gpurun_out/qlora_pf2
for r in 1 2 3; do
  for arm in pf inline lora; do
    case $arm in
      pf) envs="FTC_NF4_PREFETCH=1"; args="--model mistral-7b --method qlora";;
      inline) envs="FTC_NF4_PREFETCH=0"; args="--model mistral-7b --method qlora";;
      lora) envs="FTC_NF4_PREFETCH=1"; args="--model mistral-7b-v0.3";;
    esac
    env $envs timeout -k 10 400 python -u bench.py $args --steps 8 --warmup 3 > gpurun_out/qlora_pf2/${arm}_r$r.log 2>&1 || { tail -5 gpurun_out/qlora_pf2/${arm}_r$r.log; exit 1; }
    echo "$arm r$r $(grep '^{' gpurun_out/qlora_pf2/${arm}_r$r.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("peak_mem_gb"))')"
  done
done
bash tools/pmc_run.sh gemm_r4 --labels gpurun_out/pmc_gemm_labels.json --match Cijk,gemm_nt -- python3 tools/pmc_gemms.py --iters 4 --ours > gpurun_out/pmc_gemm_r4.log 2>&1; rc=$?; tail -25 gpurun_out/pmc_gemm_r4.md 2>/dev/null | cut -c1-200; exit $rc
