#!/bin/bash
# PMC counters for the flash-attention kernels (own runs, kernel-trace only; see guide §7).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out/pmc
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
           "SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $R/gpurun_out/pmc/p$i -o attn \
     -- python3 $R/tools/bench_attention.py --rounds 1 --iters 2 > $R/gpurun_out/pmc/p$i.log 2>&1) || { echo "pass $i failed"; tail -5 $R/gpurun_out/pmc/p$i.log; exit 1; }
done
find gpurun_out/pmc -name "*counter_collection.csv" | head
