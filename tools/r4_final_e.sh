#!/bin/bash
# final tree: full GPU suite + smoke + the driver's bench command
set -o pipefail
mkdir -p gpurun_out/final_e
bash tools/r4_gpu_suite.sh || exit 1
cp gpurun_out/pytest_gpu_full.log gpurun_out/smoke.log gpurun_out/final_e/
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_e/driver_cmd.log 2>&1 || { tail -20 gpurun_out/final_e/driver_cmd.log; exit 1; }
grep '^{' gpurun_out/final_e/driver_cmd.log | tail -1 | cut -c1-200
