#!/bin/bash
# A/B of the packed-fp32 softmax arithmetic in the flash kernels (FWD_PK_SOFTMAX: forward scale / shift
# and row sum as v_pk_fma_f32 / v_pk_add_f32; BWD_PK_EXP: the dQ pass's scale / shift).
#   bash tools/pk_softmax_ab.sh build   (CPU, after the in-tree build): ab_nopk/ = a copy of the package
#                                       whose _C.so has both flash files built with the knobs at 0
# Result (profiles/r3/pk_softmax/, one box, knobs at 1 in the tree): forward 0.605 / 0.615 vs 0.589 /
# 0.578 ms, headline 35,376 / 35,429 vs 35,533 / 35,527 tok/s -> the packed form is slower; both knobs
# default to 0 (to rerun: build the tree with them at 1)
#   bash tools/pk_softmax_ab.sh run     (GPU box): numerics of the variant, interleaved attention timings
#                                       and headline steps of both trees
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
V=ab_nopk
if [ "$1" = "build" ]; then
  TL=$(python -c 'import torch,os;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
  rm -rf $V; mkdir -p $V/obj $V/tools
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c csrc/kernels/flash_attn_fwd.hip -o $V/obj/flash_attn_fwd.hip.o \
    -I csrc/kernels -ffp-contract=fast -Wno-unused-result -DFWD_PK_SOFTMAX=0 || exit 1
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c csrc/kernels/flash_attn_bwd.hip -o $V/obj/flash_attn_bwd.hip.o \
    -I csrc/kernels -ffp-contract=fast -Wno-unused-result -DBWD_PK_EXP=0 || exit 1
  objs=""; for o in build/native/*.hip.o; do b=$(basename $o); [ -f $V/obj/$b ] && objs="$objs $V/obj/$b" || objs="$objs $o"; done
  cp -r finetune_controller_amd tests bench.py pytest.ini $V/ && cp tools/bench_attention.py $V/tools/ && rm $V/finetune_controller_amd/_C.so
  find $V -name __pycache__ -prune -exec rm -rf {} +
  hipcc --offload-arch=gfx950 -shared -fPIC -o $V/finetune_controller_amd/_C.so $objs build/native/binding.cpp.o -L$TL -lc10 \
    -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -Wl,-rpath,$TL -L/opt/rocm/lib -lamdhip64 || exit 1
  rm -rf $V/obj
  echo "built $V"
  exit 0
fi
O=gpurun_out/pk_softmax; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "flash or rope or llama_hip_vs_fp32" > $O/pytest_tree.log 2>&1 || { tail -5 $O/pytest_tree.log; exit 1; }
echo "tree: $(tail -1 $O/pytest_tree.log)"
for r in 1 2; do
  timeout -k 10 300 python tools/bench_attention.py --rounds 3 > $O/attn_pk$r.log 2>&1 || exit 1
  (cd $V && timeout -k 10 300 python tools/bench_attention.py --rounds 3 > ../$O/attn_nopk$r.log 2>&1) || exit 1
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_pk$r.json 2>/dev/null || exit 1
  (cd $V && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > ../$O/bench_nopk$r.json 2>/dev/null) || exit 1
done
