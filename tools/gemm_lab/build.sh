#!/bin/bash
# Build the GEMM lab kernels (CPU-side, in-tree; the .so files travel to the GPU box with the snapshot), each
# variant in its own library (no co-compiled variants): libgemm_pp_d{0..3}.so -- the ping-pong kernel with
# its DMA pieces after / before the fragment reads, half / all of them inside the next compute phase;
# libgemm_pp_m{1,2,3}.so -- timing-only ablations of d0 (wrong results): no loop DMA / no loop DMA + reads /
# no counted waits.
set -e
cd "$(dirname "$0")/../.."
build() { hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Icsrc/kernels -ffp-contract=fast "$@"; }
for d in 0 1 2 3; do build -DPPM=0 -DDMAP=$d tools/gemm_lab/gemm_pp.hip -o tools/gemm_lab/libgemm_pp_d$d.so & done
for m in 1 2 3; do build -DPPM=$m -DDMAP=0 tools/gemm_lab/gemm_pp.hip -o tools/gemm_lab/libgemm_pp_m$m.so & done
wait
# the hand-written projection (NT, with the RoPE epilogue) and weight-gradient (TN) GEMMs: lab-only since
# round 6 (they never beat hipBLASLt on a shipped shape; tools/gemm_lab/lab.py loads this library)
build tools/gemm_lab/gemm_nt.hip tools/gemm_lab/gemm_tn.hip -o tools/gemm_lab/libgemm_lab.so
