#!/bin/bash
# Sustained throughput: the flagship LoRA step (bench config) for 400 steps through the training CLI,
# logging tokens/s every 20 steps, then the driver's default bench right after (thermally soaked chip).
# Usage on the GPU box: bash tools/sustained.sh   -> gpurun_out/sustained/
O=gpurun_out/sustained
mkdir -p $O
timeout -k 10 420 python -u -m finetune_controller_amd.train.cli --model llama3-8b --method lora --batch-size 4 \
  --seq-len 4096 --synthetic --max-steps 400 --log-interval 20 --warmup-steps 10 --no-resume \
  --checkpoint-path $O/ck > $O/train400.log 2>&1 || exit 1
rm -rf $O/ck/*.safetensors $O/ck/*.pt
timeout -k 10 300 python -u bench.py > $O/bench_after.json 2> $O/bench_after.err
