#!/bin/bash
# same-box A/B: LoRA headline step, tree before today's stream-kernel changes (.ab_base) vs HEAD
# (historical record of a measurement: the A/B switch or worktree it used was removed afterwards; see profiles/r4/)
set -o pipefail
mkdir -p gpurun_out/ab17
for r in 1 2; do
  (cd .ab_base && timeout -k 10 400 python -u bench.py --steps 10 --warmup 3) > gpurun_out/ab17/base_$r.log 2>&1 || { tail -5 gpurun_out/ab17/base_$r.log; exit 1; }
  grep '^{' gpurun_out/ab17/base_$r.log | cut -c1-160
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ab17/head_$r.log 2>&1 || { tail -5 gpurun_out/ab17/head_$r.log; exit 1; }
  grep '^{' gpurun_out/ab17/head_$r.log | cut -c1-160
done
