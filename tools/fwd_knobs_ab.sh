#!/bin/bash
# A/B of the flash forward's build-time knobs (FWD_KPRE: K-fragment reads issued ahead of the S MFMA
# chain, default 4; FWD_PRIO: s_setprio(1) over the S MFMA phase, default 0).
#   bash tools/fwd_knobs_ab.sh build    (CPU, after `python -m finetune_controller_amd.tools.build`):
#        ab_fwd_<name>/ = a copy of the package whose _C.so has flash_attn_fwd built with the knob
#   bash tools/fwd_knobs_ab.sh run      (GPU box): numerics of each variant, interleaved timings
# Result (profiles/r2/fwd_knobs/, one box): base 0.560 / 0.564 ms, prio 0.574 / 0.570 (slower: the
# raised priority starves the partner wave's softmax), kpre8 0.564 / 0.567, kpre2 0.563 / 0.559 (noise)
# -> the defaults (KPRE 4, no priority) stay.
# narrow (8-byte O stores instead of the 16-byte epilogue, profiles/r2/fwd_wide_store/): 0.559-0.562 vs
# 0.553-0.555 ms, headline 36,752 / 36,818 vs 36,918 / 36,822 tok/s -> wide stores are the default.
# FWD_EARLY_DMA=1 (tile 0's DMA before the Q loads; profiles/r2/fwd_early_dma/, 'base' = early there):
# 0.586 / 0.566 vs 0.581 / 0.571 ms, headline 36,307 / 36,322 vs 36,306 / 36,302 -> noise, stays off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
declare -A FLAGS=([prio]="-DFWD_PRIO=1" [kpre8]="-DFWD_KPRE=8" [kpre2]="-DFWD_KPRE=2" [narrow]="-DFWD_WIDE_STORE=0" [lateq]="-DFWD_EARLY_DMA=0")
# variants to build / run (default: the latest question); e.g. FWD_AB_NAMES="prio kpre8 kpre2"
read -r -a NAMES <<< "${FWD_AB_NAMES:-lateq}"
if [ "$1" = "build" ]; then
  TL=$(python -c 'import torch,os;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
  for n in "${NAMES[@]}"; do
    V=ab_fwd_$n; rm -rf $V; mkdir -p $V/obj $V/tools
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c csrc/kernels/flash_attn_fwd.hip -o $V/obj/flash_attn_fwd.hip.o \
      -I csrc/kernels -Wno-unused-result ${FLAGS[$n]} || exit 1
    objs=""; for o in build/native/*.hip.o; do b=$(basename $o); [ -f $V/obj/$b ] && objs="$objs $V/obj/$b" || objs="$objs $o"; done
    cp -r finetune_controller_amd tests bench.py pytest.ini $V/ && cp tools/bench_attention.py $V/tools/ && rm $V/finetune_controller_amd/_C.so
    find $V -name __pycache__ -prune -exec rm -rf {} +
    hipcc --offload-arch=gfx950 -shared -fPIC -o $V/finetune_controller_amd/_C.so $objs build/native/binding.cpp.o -L$TL -lc10 \
      -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -Wl,-rpath,$TL -L/opt/rocm/lib -lamdhip64 || exit 1
    rm -rf $V/obj
    echo "built $V"
  done
  exit 0
fi
O=gpurun_out/fwd_knobs; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "flash or llama_lora or packed or tail or family or gpt2 or decode or generate" > $O/pytest_tree.log 2>&1 \
  || { tail -5 $O/pytest_tree.log; exit 1; }
echo "tree: $(tail -1 $O/pytest_tree.log)"
for n in "${NAMES[@]}"; do
  (cd ab_fwd_$n && timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "flash or llama_lora or packed or tail" > ../$O/pytest_$n.log 2>&1) \
    || { tail -5 $O/pytest_$n.log; exit 1; }
  echo "$n: $(tail -1 $O/pytest_$n.log)"
done
for r in 1 2; do
  timeout -k 10 300 python tools/bench_attention.py --rounds 3 > $O/attn_base$r.log 2>&1 || exit 1
  echo "base  $(grep -v amdgpu $O/attn_base$r.log | tail -1 | grep -o "\"ours_fwd\": {[^}]*}")"
  for n in "${NAMES[@]}"; do
    (cd ab_fwd_$n && timeout -k 10 300 python tools/bench_attention.py --rounds 3 > ../$O/attn_$n$r.log 2>&1) || exit 1
    echo "$n $(grep -v amdgpu $O/attn_$n$r.log | tail -1 | grep -o "\"ours_fwd\": {[^}]*}")"
  done
done
for r in 1 2; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_base$r.log 2>&1 || exit 1
  echo "base $(grep '^{' $O/bench_base$r.log | cut -c70-140)"
  for n in "${NAMES[@]}"; do
    (cd ab_fwd_$n && timeout -k 10 400 python bench.py --steps 10 --warmup 3 > ../$O/bench_$n$r.log 2>&1) || exit 1
    echo "$n $(grep '^{' $O/bench_$n$r.log | cut -c70-140)"
  done
done
