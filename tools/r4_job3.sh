#!/bin/bash
# QB2 forward: numerics first (small shapes), then the variant bench; GEMM stamps; full suite + smoke
set -o pipefail
mkdir -p gpurun_out/attn_r4 gpurun_out/gemm_r4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" > gpurun_out/attn_r4/pytest_flash.log 2>&1; rc=$?; tail -3 gpurun_out/attn_r4/pytest_flash.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_attn_fwd.py > gpurun_out/attn_r4/fwd_qb.log 2>&1; rc=$?; cat gpurun_out/attn_r4/fwd_qb.log | grep "^{"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/gemm_lab/stamps.py > gpurun_out/gemm_r4/stamps.log 2>&1; echo "stamps rc=$?"; grep "^{" gpurun_out/gemm_r4/stamps.log
bash tools/r4_gpu_suite.sh
