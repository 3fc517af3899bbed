#!/bin/bash
# one-shot grids for the element-wise stream kernels: tests, per-op A/B, full-FT A/B
# (historical record of a measurement: the A/B switch or worktree it used was removed afterwards; see profiles/r4/)
set -o pipefail
mkdir -p gpurun_out/oneshot
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "swiglu or rope or splitk or nf4 or wgrad_split or adamw" > gpurun_out/oneshot/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/oneshot/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for p in 0 1; do
    FTC_ONESHOT=$p TAG=oneshot$p timeout -k 10 300 python -u tools/bench_stream_ops.py >> gpurun_out/oneshot/ops.log 2>&1 || { tail -5 gpurun_out/oneshot/ops.log; exit 1; }
  done
done
grep '^{' gpurun_out/oneshot/ops.log
for p in 0 1; do
  FTC_ONESHOT=$p timeout -k 10 500 python -u bench.py --method full --steps 10 --warmup 3 > gpurun_out/oneshot/full_$p.log 2>&1 || { tail -5 gpurun_out/oneshot/full_$p.log; exit 1; }
  grep '^{' gpurun_out/oneshot/full_$p.log | cut -c1-200
done
