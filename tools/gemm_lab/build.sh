#!/bin/bash
# Build the GEMM lab kernels (CPU-side, in-tree; the .so files travel to the GPU box with the snapshot):
# libgemm_pp.so (the kernel) and libgemm_pp_m{1,2,3}.so (timing-only ablations, wrong results: no loop DMA /
# no loop DMA + fragment reads / no counted waits) -- each in its own library (no co-compiled variants).
set -e
cd "$(dirname "$0")/../.."
for m in 0 1 2 3; do
  out=tools/gemm_lab/libgemm_pp.so; [ $m -gt 0 ] && out=tools/gemm_lab/libgemm_pp_m$m.so
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Icsrc/kernels -ffp-contract=fast -DPPM=$m \
    tools/gemm_lab/gemm_pp.hip -o $out &
done
wait
