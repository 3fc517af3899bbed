#!/bin/bash
# Per-kernel times of the flash backward variants (FTC_FLASH_DKDV_WAVES=4|8) + a counter list.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/dkdv
for v in ${VARIANTS:-4 8}; do
  (cd /tmp && FTC_FLASH_DKDV_WAVES=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $R/gpurun_out/dkdv/$v -o attn -- python3 $R/tools/bench_attention.py --rounds 1 --iters 5 \
     > $R/gpurun_out/dkdv/$v.log 2>&1) || { echo "variant $v failed"; tail -5 $R/gpurun_out/dkdv/$v.log; exit 1; }
  f=$(find gpurun_out/dkdv/$v -name "*kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "dkdv|dq_kernel|flash_fwd" "$f" | cut -d, -f1-4
done
(cd /tmp && timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/dkdv/counters.txt 2>&1) || true
