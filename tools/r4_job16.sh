#!/bin/bash
# one-shot RMSNorm / delta launches: tests, RMSNorm A/B, LoRA step kernel table
# (historical record of a measurement: the A/B switch or worktree it used was removed afterwards; see profiles/r4/)
set -o pipefail
mkdir -p gpurun_out/oneshot2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "rmsnorm or flash or norm" > gpurun_out/oneshot2/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/oneshot2/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for p in 0 1; do
    echo "FTC_RMS_ONESHOT=$p" >> gpurun_out/oneshot2/rms.log
    FTC_RMS_ONESHOT=$p timeout -k 10 300 python -u tools/bench_rmsnorm.py >> gpurun_out/oneshot2/rms.log 2>&1 || { tail -5 gpurun_out/oneshot2/rms.log; exit 1; }
  done
done
grep -v "^{\"kernel\": \"tail" gpurun_out/oneshot2/rms.log
for p in 0 1; do
  FTC_RMS_ONESHOT=$p timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/oneshot2/lora_$p.log 2>&1 || { tail -5 gpurun_out/oneshot2/lora_$p.log; exit 1; }
  grep '^{' gpurun_out/oneshot2/lora_$p.log | cut -c1-200
done
