#!/bin/bash
# A/B: flash kernels compiled with vs without SLP vectorization (packed f32 VALU beside MFMAs).
# ab_noslp/ holds a copy of the package whose _C.so has flash_attn_{fwd,bwd} built with -fno-slp-vectorize
# (built here first if absent; run `python -m finetune_controller_amd.tools.build` before).
# Result (profiles/r2/noslp/): neutral -- fwd 0.581/0.588 vs 0.582/0.586 ms, LoRA step 36.71/36.57k vs 36.61/36.46k.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/noslp; mkdir -p $O
if [ ! -f ab_noslp/finetune_controller_amd/_C.so ]; then  # build the variant (CPU-only step)
  V=ab_noslp; mkdir -p $V/obj $V/tools
  for f in fwd bwd; do
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c csrc/kernels/flash_attn_$f.hip -o $V/obj/flash_attn_$f.hip.o \
      -I csrc/kernels -Wno-unused-result -ffp-contract=fast -fno-slp-vectorize || exit 1
  done
  objs=""; for o in build/native/*.hip.o; do b=$(basename $o); [ -f $V/obj/$b ] && objs="$objs $V/obj/$b" || objs="$objs $o"; done
  TL=$(python -c 'import torch,os;print(os.path.join(os.path.dirname(torch.__file__),"lib"))')
  cp -r finetune_controller_amd tests bench.py pytest.ini $V/ && cp tools/bench_attention.py $V/tools/ && rm $V/finetune_controller_amd/_C.so
  hipcc --offload-arch=gfx950 -shared -fPIC -o $V/finetune_controller_amd/_C.so $objs build/native/binding.cpp.o -L$TL -lc10 \
    -lc10_hip -ltorch -ltorch_cpu -ltorch_hip -ltorch_python -Wl,-rpath,$TL -L/opt/rocm/lib -lamdhip64 || exit 1
fi
(cd ab_noslp && timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or llama_lora or packed" \
  > ../$O/pytest.log 2>&1) || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python tools/bench_attention.py --rounds 3 > $O/attn_base$r.log 2>&1 || exit 1
  echo "base  $(grep -v amdgpu $O/attn_base$r.log | tail -1 | cut -c1-260)"
  (cd ab_noslp && timeout -k 10 300 python tools/bench_attention.py --rounds 3 > ../$O/attn_noslp$r.log 2>&1) || exit 1
  echo "noslp $(grep -v amdgpu $O/attn_noslp$r.log | tail -1 | cut -c1-260)"
done
for r in 1 2; do
  timeout -k 10 400 python bench.py --steps 8 --warmup 2 > $O/bench_base$r.log 2>&1 || exit 1
  echo "bench base  $(grep '^{' $O/bench_base$r.log | cut -c80-140)"
  (cd ab_noslp && timeout -k 10 400 python bench.py --steps 8 --warmup 2 > ../$O/bench_noslp$r.log 2>&1) || exit 1
  echo "bench noslp $(grep '^{' $O/bench_noslp$r.log | cut -c80-140)"
done
