#!/bin/bash
# LAB (round 5): NF4 decode rewrite and QLoRA step (old vs new extension), CE chunk rows on the headline,
# attention counters of the current build.  -> gpurun_out/r5f/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/r5f; mkdir -p $O
P=finetune_controller_amd
cp $P/_C.so $P/_C_new.so
for r in 1 2; do
  for v in a new; do
    cp $P/_C_$v.so $P/_C.so
    timeout -k 10 120 python -u tools/bench_attention.py --rounds 5 > $O/attn_${v}_r$r.log 2>&1 || { tail $O/attn_${v}_r$r.log; exit 1; }
    echo "$v r$r attn: $(grep -h '^{' $O/attn_${v}_r$r.log | cut -c90-200)"
    timeout -k 10 120 python -u tools/bench_nf4_decode.py > $O/nf4_${v}_r$r.log 2>&1 || { tail $O/nf4_${v}_r$r.log; exit 1; }
    timeout -k 10 300 python -u bench.py --model mistral-7b --method qlora > $O/qlora_${v}_r$r.log 2>&1 || { tail $O/qlora_${v}_r$r.log; exit 1; }
    echo "$v r$r qlora: $(grep -h '^{' $O/qlora_${v}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
cp $P/_C_new.so $P/_C.so
for r in 1 2; do
  for c in 4096 16384; do
    timeout -k 10 300 python -u bench.py --ce-chunk-rows $c > $O/ce${c}_r$r.log 2>&1 || { tail $O/ce${c}_r$r.log; exit 1; }
    echo "ce $c r$r: $(grep -h '^{' $O/ce${c}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["peak_mem_gb"])')"
  done
done
bash tools/pmc_run.sh attn_r5 -- python3 tools/bench_attention.py --rounds 1 --iters 2 > $O/pmc_attn.log 2>&1 || { tail $O/pmc_attn.log; exit 1; }
cp gpurun_out/pmc_attn_r5.md $O/
head -12 $O/pmc_attn_r5.md
