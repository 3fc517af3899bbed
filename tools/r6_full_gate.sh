#!/bin/bash
# VERDICT r5 Next #6: full FT with the HBM-bound backward kernels gated behind the side-stream dW
# (FTC_DW_GATE=1) vs the current overlap, same box, alternating; LoRA control; kernel tables of both.
# -> gpurun_out/r6_full_gate/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/r6_full_gate; mkdir -p $O
val() { grep -h '"metric"' "$1" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/lora_control.log 2>&1 || { tail $O/lora_control.log; exit 1; }
echo "lora control: $(val $O/lora_control.log)"
for r in 1 2; do
  for g in 0 1; do
    FTC_DW_GATE=$g timeout -k 10 400 python -u bench.py --method full --steps 10 --warmup 3 > $O/full_gate${g}_$r.log 2>&1 \
      || { tail $O/full_gate${g}_$r.log; exit 1; }
    echo "full gate=$g r$r: $(val $O/full_gate${g}_$r.log)"
  done
done
for g in 0 1; do
  FTC_DW_GATE=$g bash tools/prof_bench.sh full_gate$g --method full --steps 3 --warmup 2 > /dev/null || exit 1
  cp gpurun_out/prof_full_gate$g.md $O/
  head -24 $O/prof_full_gate$g.md | tail -18
done
