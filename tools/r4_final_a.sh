#!/bin/bash
# round-4 tree: full GPU suite + smoke, the driver's bench command (twice), LoRA and full-FT kernel tables
set -o pipefail
mkdir -p gpurun_out/final
bash tools/r4_gpu_suite.sh || exit 1
cp gpurun_out/pytest_gpu_full.log gpurun_out/smoke.log gpurun_out/final/
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/driver_cmd_r$r.log 2>&1 || { tail -20 gpurun_out/final/driver_cmd_r$r.log; exit 1; }
  grep '^{' gpurun_out/final/driver_cmd_r$r.log | tail -1 | cut -c1-220
done
bash tools/prof_bench.sh lora_r4 --steps 3 --warmup 2 > /dev/null || exit 1
head -14 gpurun_out/prof_lora_r4.md
timeout -k 10 500 python -u bench.py --method full --steps 8 --warmup 3 > gpurun_out/final/full.log 2>&1 || { tail -20 gpurun_out/final/full.log; exit 1; }
grep '^{' gpurun_out/final/full.log | tail -1 | cut -c1-200
