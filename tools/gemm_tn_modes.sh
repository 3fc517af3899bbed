#!/bin/bash
# A/B of the weight-gradient GEMM variants (csrc/kernels/gemm_tn.hip) on one box (results are wrong in
# modes 2 / 8 -- timing only): FTC_GEMM_TN_WAVES 4 | 8; FTC_GEMM_TN_MODE 0 normal, 2 no DMA (compute
# ceiling), 8 DMA always of K-step 0 (L2-resident); FTC_GEMM_TN_GROUP = M-blocks per tile group
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python tools/bench_gemm_tn.py --shapes ${SHAPES:-gu,down} --cdtype bf16 \
    > gpurun_out/gemm_tn_$tag.log 2>&1 || exit 1
  grep '^{' gpurun_out/gemm_tn_$tag.log | sed "s/^/$tag /" | cut -c1-140
}
run w8m0 FTC_GEMM_TN_WAVES=8
run w8m8 FTC_GEMM_TN_WAVES=8 FTC_GEMM_TN_MODE=8
run w8g1 FTC_GEMM_TN_WAVES=8 FTC_GEMM_TN_GROUP=1
run w8g2 FTC_GEMM_TN_WAVES=8 FTC_GEMM_TN_GROUP=2
run w8g8 FTC_GEMM_TN_WAVES=8 FTC_GEMM_TN_GROUP=8
run w8g16 FTC_GEMM_TN_WAVES=8 FTC_GEMM_TN_GROUP=16
run w4m8 FTC_GEMM_TN_WAVES=4 FTC_GEMM_TN_MODE=8
