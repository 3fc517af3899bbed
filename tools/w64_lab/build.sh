#!/bin/bash
# Build variants of the flash forward (csrc/kernels/flash_attn_fwd.hip) as standalone ctypes libraries for
# one-call GPU A/B and numerics experiments: tools/w64_lab/lib<name>.so (extern "C" ftc_flash_fwd*).
# Timing-only ablations (wrong results): W64_ABL_NOBAR / NODMA / NOEXP / NOLDS (see the source).
set -e
cd "$(dirname "$0")/../.."
b() { n=$1; shift; hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Icsrc/kernels -ffp-contract=fast \
      -mllvm -amdgpu-mfma-vgpr-form -fno-slp-vectorize -DW64_LAB=1 "$@" csrc/kernels/flash_attn_fwd.hip -o tools/w64_lab/lib$n.so; }
b base &
b abl_nolds -DW64_ABL_NOLDS=1 &
b abl_nolds_noexp -DW64_ABL_NOLDS=1 -DW64_ABL_NOEXP=1 &
b abl_all4 -DW64_ABL_NOLDS=1 -DW64_ABL_NOEXP=1 -DW64_ABL_NODMA=1 -DW64_ABL_NOBAR=1 &

b stamps -DW64_STAMPS=1 &
b v3ring -DW64_V3=1 -DW64_SEAM=0 &
b w32pin -DFWD_PIN=1 &
wait
