#!/bin/bash
# LAB: flash-backward variants (fused delta in dQ | separate delta pass | dS spill) on one GPU -> gpurun_out/attn_ab2/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/attn_ab2; mkdir -p $O
export TMPDIR=/tmp
for m in sep ds; do
  FTC_FLASH_BWD_MODE=$m timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_kernels_gpu.py -k "flash_attention_fwd_bwd or flash_bwd_rope or llama3_8b" > $O/pytest_$m.log 2>&1 \
    || { tail -30 $O/pytest_$m.log; exit 1; }
  tail -1 $O/pytest_$m.log
done
timeout -k 10 180 python -u tools/bench_attention.py --ab sep,ds --rounds 7 > $O/bench_b4.log 2>&1 || { tail $O/bench_b4.log; exit 1; }
grep shape $O/bench_b4.log
for m in fused sep ds; do
  FTC_FLASH_BWD_MODE=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_$m -o k -- \
    python3 tools/bench_attention.py --rounds 1 --iters 5 > $O/prof_$m.log 2>&1 || { tail $O/prof_$m.log; exit 1; }
done
for r in 1 2; do
  for m in fused sep; do
    FTC_FLASH_BWD_MODE=$m timeout -k 10 300 python -u bench.py > $O/bench_${m}_$r.log 2>&1 || { tail $O/bench_${m}_$r.log; exit 1; }
    echo "$m r$r: $(grep -h '"metric"' $O/bench_${m}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
