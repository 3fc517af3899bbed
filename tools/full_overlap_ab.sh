#!/bin/bash
# Full fine-tuning A/B: optimizer update overlapped with the next forward (FTC_OPT_OVERLAP=1, opt-in)
# vs serial, interleaved on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for t in 1 0 1 0; do
  FTC_OPT_OVERLAP=$t timeout -k 10 400 python bench.py --method full --steps 6 --warmup 2 ${EXTRA:-} > gpurun_out/full_overlap_$t.log 2>&1 || exit 1
  echo "FTC_OPT_OVERLAP=$t $(grep '^{' gpurun_out/full_overlap_$t.log | cut -c80-160)"
done
