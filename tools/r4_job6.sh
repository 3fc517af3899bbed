#!/bin/bash
# flash: QB2 forward + IL dK/dV numerics (every flash test runs qb1 / qb2 / il), then both variant benches;
# split-K weight gradients; GEMM cache-policy sweep
set -o pipefail
mkdir -p gpurun_out/attn_r4 gpurun_out/dw_r4
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or wgrad_split" > gpurun_out/attn_r4/pytest_flash6.log 2>&1; rc=$?; tail -3 gpurun_out/attn_r4/pytest_flash6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_attn_fwd.py > gpurun_out/attn_r4/fwd_qb6.log 2>&1; rc=$?; grep "^{" gpurun_out/attn_r4/fwd_qb6.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_attn_bwd.py > gpurun_out/attn_r4/bwd_il6.log 2>&1; rc=$?; grep "^{" gpurun_out/attn_r4/bwd_il6.log; [ $rc -eq 0 ] || exit $rc
FTC_DW_SPLIT=auto timeout -k 10 300 python -u tools/bench_dw_split.py > gpurun_out/dw_r4/split.log 2>&1; rc=$?; grep "^{" gpurun_out/dw_r4/split.log; [ $rc -eq 0 ] || exit $rc
bash tools/r4_job4.sh
