#!/bin/bash
# dK/dV: asm DMA in the 8-wave kernel (no phase-A drain) + IL fixes -- numerics, bench, stamps
set -o pipefail
mkdir -p gpurun_out/attn_r4
timeout -k 5 60 ./tools/check_il_11 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" > gpurun_out/attn_r4/pytest_flash9.log 2>&1; rc=$?; tail -2 gpurun_out/attn_r4/pytest_flash9.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_attn_bwd.py > gpurun_out/attn_r4/bwd_il9.log 2>&1; rc=$?; grep "^{" gpurun_out/attn_r4/bwd_il9.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/stamp_dkdv 0 > gpurun_out/attn_r4/stamp8_9.log 2>&1 && sed -n 1,6p gpurun_out/attn_r4/stamp8_9.log && FTC_FLASH_DKDV_WAVES=il timeout -k 10 120 ./tools/stamp_dkdv 0 > gpurun_out/attn_r4/stamp_il9.log 2>&1 && sed -n 1,4p gpurun_out/attn_r4/stamp_il9.log
