#!/bin/bash
# Full fine-tuning A/B of the weight-gradient path: FTC_GEMM_TN = 0 (hipBLASLt on transposed copies of
# x for every projection) vs auto (hand-written TN GEMM for the wide down-projection input), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for t in 0 auto 0 auto; do
  FTC_GEMM_TN=$t timeout -k 10 400 python bench.py --method full --steps 6 --warmup 2 > gpurun_out/full_gemm_tn_$t.log 2>&1 || exit 1
  echo "FTC_GEMM_TN=$t $(grep '^{' gpurun_out/full_gemm_tn_$t.log | cut -c80-150)"
done
