#!/bin/bash
# AdamW wide kernel: bitwise tests + A/B at 2e9 elements
# (historical record of a measurement: the A/B switch or worktree it used was removed afterwards; see profiles/r4/)
set -o pipefail
mkdir -p gpurun_out/adamw
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adamw" > gpurun_out/adamw/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/adamw/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_adamw.py > gpurun_out/adamw/ab.log 2>&1; rc=$?; cat gpurun_out/adamw/ab.log; [ $rc -eq 0 ] || exit $rc
N=8.03e9 timeout -k 10 400 python -u tools/bench_adamw.py > gpurun_out/adamw/ab_8b.log 2>&1; rc=$?; cat gpurun_out/adamw/ab_8b.log; exit $rc
