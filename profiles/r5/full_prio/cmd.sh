#!/bin/bash
# LAB: full fine-tuning with the main stream on a high-priority HIP queue (side-stream dW at normal priority)
# vs the default and the serial path; LoRA kernel table of the current build.  -> gpurun_out/full_prio/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
out=gpurun_out/full_prio; mkdir -p $out
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "flash or llama3_8b" > $out/pytest_flash.log 2>&1 || { tail -30 $out/pytest_flash.log; exit 1; }
tail -1 $out/pytest_flash.log
FTC_LAB_PRIO=1 bash tools/prof_bench.sh full_prio --method full --steps 3 --warmup 2 > /dev/null || exit 1
cp gpurun_out/prof_full_prio.md $out/
for r in 1 2; do
  for mode in def prio ser; do
    case $mode in def) env="";; prio) env="FTC_LAB_PRIO=1";; ser) env="FTC_DW_STREAM=0";; esac
    env $env timeout -k 10 400 python bench.py --method full --steps 10 --warmup 3 > $out/full_${mode}_r$r.log 2>&1 || exit 1
    echo "full $mode r$r: $(grep '^{' $out/full_${mode}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
bash tools/prof_bench.sh lora_r5b --steps 3 --warmup 2 > /dev/null || exit 1
cp gpurun_out/prof_lora_r5b.md $out/
head -14 $out/prof_lora_r5b.md | tail -10 | cut -c1-150
