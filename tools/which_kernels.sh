#!/bin/bash
# kernel names actually dispatched by the attention bench under a given env (rocprofv3 kernel trace)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/which
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/which -o w \
   -- python3 $R/tools/bench_attention.py --rounds 1 --iters 3 > $R/gpurun_out/which/w.log 2>&1) || exit 1
tail -1 gpurun_out/which/w.log
cut -d, -f1-4 gpurun_out/which/w_kernel_stats.csv | grep -i "flash\|bwd_" | head
