#!/bin/bash
# Whole-step hipGraph A/B (bench --graph) on the headline 8B LoRA step and the 1B model (launch-bound?).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/graph_ab; mkdir -p $O
for r in 1 2; do
  for g in "" "--graph"; do
    tag=8b${g:+_graph}_$r
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 4 $g > $O/$tag.json 2> $O/$tag.err || exit 1
    echo "$tag $(cut -c80-135 $O/$tag.json)"
  done
done
for g in "" "--graph"; do
  tag=1b${g:+_graph}
  timeout -k 10 300 python -u bench.py --model llama3.2-1b --steps 20 --warmup 4 $g > $O/$tag.json 2> $O/$tag.err || exit 1
  echo "$tag $(cut -c80-135 $O/$tag.json)"
done
