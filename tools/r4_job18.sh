#!/bin/bash
# full FT: W^T refresh eager (after AdamW) vs lazy (inside the next backward), same box, two rounds
# (historical record of a measurement: the A/B switch or worktree it used was removed afterwards; see profiles/r4/)
set -o pipefail
mkdir -p gpurun_out/wt_eager
for r in 1 2; do
  for e in 0 1; do
    FTC_WT_EAGER=$e timeout -k 10 500 python -u bench.py --method full --steps 10 --warmup 3 > gpurun_out/wt_eager/full_e${e}_r$r.log 2>&1 || { tail -5 gpurun_out/wt_eager/full_e${e}_r$r.log; exit 1; }
    echo "eager=$e r=$r $(grep '^{' gpurun_out/wt_eager/full_e${e}_r$r.log | cut -c80-190)"
  done
done
