#!/bin/bash
# LAB: full fine-tuning with the side-stream weight gradients confined to a CU subset
# (hipExtStreamCreateWithCUMask) vs the unmasked side stream.  -> gpurun_out/full_cumask/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
out=gpurun_out/full_cumask; mkdir -p $out
for r in 1 2; do
  for m in none stride:4 stride:2 block:64 stride:8; do
    tag=${m/:/}
    if [ $m = none ]; then env=""; else env="FTC_LAB_DW_CUMASK=$m"; fi
    env $env timeout -k 10 300 python bench.py --method full --steps 8 --warmup 3 > $out/full_${tag}_r$r.log 2>&1 || { tail $out/full_${tag}_r$r.log; exit 1; }
    echo "full $m r$r: $(grep '^{' $out/full_${tag}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
