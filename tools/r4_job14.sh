#!/bin/bash
# one-shot AdamW: kernel tests, throughput, full-FT bench (the step whose optimizer it is)
set -o pipefail
mkdir -p gpurun_out/adamw
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adamw or zero1 or optim" > gpurun_out/adamw/pytest2.log 2>&1; rc=$?; tail -3 gpurun_out/adamw/pytest2.log; [ $rc -eq 0 ] || exit $rc
N=8.03e9 timeout -k 10 300 python -u tools/bench_adamw.py > gpurun_out/adamw/oneshot_8b.log 2>&1; rc=$?; cat gpurun_out/adamw/oneshot_8b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --method full --steps 10 --warmup 3 > gpurun_out/adamw/full.log 2>&1; rc=$?; grep '^{' gpurun_out/adamw/full.log | cut -c1-220; exit $rc
