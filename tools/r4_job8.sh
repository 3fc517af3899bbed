#!/bin/bash
# IL dK/dV iteration: numerics (flash tests), bwd bench, stamps
set -o pipefail
mkdir -p gpurun_out/attn_r4
for b in 10 11; do timeout -k 5 60 ./tools/check_il_$b || exit 1; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash" > gpurun_out/attn_r4/pytest_flash8.log 2>&1; rc=$?; tail -2 gpurun_out/attn_r4/pytest_flash8.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/bench_attn_bwd.py > gpurun_out/attn_r4/bwd_il8.log 2>&1; rc=$?; grep "^{" gpurun_out/attn_r4/bwd_il8.log; [ $rc -eq 0 ] || exit $rc
FTC_FLASH_DKDV_WAVES=il timeout -k 10 120 ./tools/stamp_dkdv 0 > gpurun_out/attn_r4/stamp_il8.log 2>&1; rc=$?; cat gpurun_out/attn_r4/stamp_il8.log; exit $rc
