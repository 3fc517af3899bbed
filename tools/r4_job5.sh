#!/bin/bash
# QB2 forward (asm DMA, pinned exp interleave): numerics + variant bench; then the GEMM M0-walk job
set -o pipefail
mkdir -p gpurun_out/attn_r4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or wgrad_split" > gpurun_out/attn_r4/pytest_flash5.log 2>&1; rc=$?; tail -3 gpurun_out/attn_r4/pytest_flash5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_attn_fwd.py > gpurun_out/attn_r4/fwd_qb5.log 2>&1; rc=$?; grep "^{" gpurun_out/attn_r4/fwd_qb5.log; [ $rc -eq 0 ] || exit $rc
bash tools/r4_job4.sh || exit $?
mkdir -p gpurun_out/dw_r4
FTC_DW_SPLIT=auto timeout -k 10 300 python -u tools/bench_dw_split.py > gpurun_out/dw_r4/split.log 2>&1; rc=$?; grep "^{" gpurun_out/dw_r4/split.log; exit $rc
