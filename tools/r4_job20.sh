#!/bin/bash
# NF4 row dequant: transposed kernel with 32-bit LDS words; tests, op A/B and Mistral-7B QLoRA A/B vs the base tree
# (historical record of a measurement: the A/B switch or worktree it used was removed afterwards; see profiles/r4/)
set -o pipefail
mkdir -p gpurun_out/nf4t
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "nf4 or qlora" > gpurun_out/nf4t/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/nf4t/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  (cd .ab_base && TAG=base timeout -k 10 300 python -u tools/bench_stream_ops.py) >> gpurun_out/nf4t/ops.log 2>&1 || { tail -5 gpurun_out/nf4t/ops.log; exit 1; }
  TAG=head timeout -k 10 300 python -u tools/bench_stream_ops.py >> gpurun_out/nf4t/ops.log 2>&1 || { tail -5 gpurun_out/nf4t/ops.log; exit 1; }
done
grep nf4 gpurun_out/nf4t/ops.log
for r in 1 2; do
  (cd .ab_base && timeout -k 10 400 python -u bench.py --model mistral-7b --method qlora --steps 8 --warmup 3) > gpurun_out/nf4t/q_base_$r.log 2>&1 || { tail -5 gpurun_out/nf4t/q_base_$r.log; exit 1; }
  echo "base $(grep '^{' gpurun_out/nf4t/q_base_$r.log | cut -c60-150)"
  timeout -k 10 400 python -u bench.py --model mistral-7b --method qlora --steps 8 --warmup 3 > gpurun_out/nf4t/q_head_$r.log 2>&1 || { tail -5 gpurun_out/nf4t/q_head_$r.log; exit 1; }
  echo "head $(grep '^{' gpurun_out/nf4t/q_head_$r.log | cut -c60-150)"
done
