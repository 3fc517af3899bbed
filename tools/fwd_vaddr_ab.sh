#!/bin/bash
# A/B: flash forward with the transposed-V read addresses hoisted out of the tile loop (tree) vs the
# previous kernel (ab_old/: a copy of the package whose _C.so was built from the previous source).
# Numerics of the tree first (flash / model GPU tests), then interleaved attention timings and bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/fwd_vaddr; mkdir -p $O
[ -f ab_old/finetune_controller_amd/_C.so ] || { echo "ab_old/ missing"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "flash or llama_lora or packed or tail or family or gpt2" > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python tools/bench_attention.py --rounds 3 > $O/attn_new$r.log 2>&1 || exit 1
  echo "new $(grep -v amdgpu $O/attn_new$r.log | tail -1 | cut -c1-260)"
  (cd ab_old && timeout -k 10 300 python tools/bench_attention.py --rounds 3 > ../$O/attn_old$r.log 2>&1) || exit 1
  echo "old $(grep -v amdgpu $O/attn_old$r.log | tail -1 | cut -c1-260)"
done
for r in 1 2; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_new$r.log 2>&1 || exit 1
  echo "new $(grep '^{' $O/bench_new$r.log | cut -c1-150)"
  (cd ab_old && timeout -k 10 400 python bench.py --steps 10 --warmup 3 > ../$O/bench_old$r.log 2>&1) || exit 1
  echo "old $(grep '^{' $O/bench_old$r.log | cut -c1-150)"
done
