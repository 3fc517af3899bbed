#!/bin/bash
# GEMM wait-segment stamps (diagnostic build) then the full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out/gemm_r4
timeout -k 10 200 python -u tools/gemm_lab/stamps.py > gpurun_out/gemm_r4/stamps.log 2>&1; echo "stamps rc=$?"; tail -8 gpurun_out/gemm_r4/stamps.log
bash tools/r4_gpu_suite.sh
