#!/bin/bash
# Full fine-tuning: the side-stream weight gradients (ops.linear, FTC_DW_STREAM, default on) against the
# serial path, with the LoRA headline as the box's clock control -- kernel tables of both (rocprofv3,
# timed steps only) and interleaved bench rounds.  -> gpurun_out/full_streams/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/full_streams; mkdir -p $out
FTC_DW_STREAM=1 bash tools/prof_bench.sh full_dws1 --method full --steps 3 --warmup 2 > /dev/null || exit 1
FTC_DW_STREAM=0 bash tools/prof_bench.sh full_dws0 --method full --steps 3 --warmup 2 > /dev/null || exit 1
cp gpurun_out/prof_full_dws1.md gpurun_out/prof_full_dws0.md $out/
for r in 1 2; do
  for d in 1 0; do
    FTC_DW_STREAM=$d timeout -k 10 400 python bench.py --method full --steps 10 --warmup 3 > $out/full_dws${d}_r$r.log 2>&1 || exit 1
    echo "full dws=$d r$r: $(grep '^{' $out/full_dws${d}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $out/lora_control.log 2>&1 || exit 1
echo "lora control: $(grep '^{' $out/lora_control.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
