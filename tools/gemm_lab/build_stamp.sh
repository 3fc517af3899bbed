#!/bin/bash
# Diagnostic build of the projection GEMM with in-kernel cycle stamps (FTC_GEMM_STAMP; never part of the
# package build): tools/gemm_lab/libgemm_stamp.so, driven by tools/gemm_lab/stamps.py through ctypes.
set -e
cd "$(dirname "$0")/../.."
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DFTC_GEMM_STAMP -I csrc/kernels -ffp-contract=fast \
  csrc/kernels/gemm_nt.hip -o tools/gemm_lab/libgemm_stamp.so
