#!/bin/bash
# A/B of the backward epilogues' 16-byte stores (BWD_WIDE_STORE=1, the tree: dK, dV and dQ rows as
# 2 x dwordx4 per 32-wide tile after a v_permlane32_swap exchange) vs 8-byte stores (narrow).
#   bash tools/bwd_store_ab.sh build   (CPU, after `python -m finetune_controller_amd.tools.build`)
#   bash tools/bwd_store_ab.sh run     (GPU box)
# Result (profiles/r2/bwd_store/, one box): backward 1.938 / 1.942 vs 1.955 / 1.964 ms narrow, headline
# 36,385 / 36,312 vs 36,258 / 36,274 tok/s -> wide stores are the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
declare -A FLAGS=([narrow]="-DBWD_WIDE_STORE=0")
NAMES=(narrow)
if [ "$1" = "build" ]; then
  TL=$(python -c 'import torch,os;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
  for n in "${NAMES[@]}"; do
    V=ab_bwd_$n; rm -rf $V; mkdir -p $V/obj $V/tools
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c csrc/kernels/flash_attn_bwd.hip -o $V/obj/flash_attn_bwd.hip.o \
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
O=gpurun_out/bwd_store; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "flash or llama_lora or packed or tail or family or gpt2" > $O/pytest_tree.log 2>&1 || { tail -5 $O/pytest_tree.log; exit 1; }
echo "tree: $(tail -1 $O/pytest_tree.log)"
for n in "${NAMES[@]}"; do
  (cd ab_bwd_$n && timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "flash or llama_lora or packed or tail" > ../$O/pytest_$n.log 2>&1) \
    || { tail -5 $O/pytest_$n.log; exit 1; }
  echo "$n: $(tail -1 $O/pytest_$n.log)"
done
for r in 1 2; do
  timeout -k 10 300 python tools/bench_attention.py --rounds 3 > $O/attn_base$r.log 2>&1 || exit 1
  echo "base  $(grep -v amdgpu $O/attn_base$r.log | tail -1 | grep -o "\"bwd_only_ms\": {[^}]*}")"
  for n in "${NAMES[@]}"; do
    (cd ab_bwd_$n && timeout -k 10 300 python tools/bench_attention.py --rounds 3 > ../$O/attn_$n$r.log 2>&1) || exit 1
    echo "$n $(grep -v amdgpu $O/attn_$n$r.log | tail -1 | grep -o "\"bwd_only_ms\": {[^}]*}")"
  done
done
for r in 1 2; do
  timeout -k 10 400 python bench.py --steps 10 --warmup 3 > $O/bench_base$r.log 2>&1 || exit 1
  echo "base $(grep '^{' $O/bench_base$r.log | cut -c70-140)"
  (cd ab_bwd_narrow && timeout -k 10 400 python bench.py --steps 10 --warmup 3 > ../$O/bench_narrow$r.log 2>&1) || exit 1
  echo "narrow $(grep '^{' $O/bench_narrow$r.log | cut -c70-140)"
done
