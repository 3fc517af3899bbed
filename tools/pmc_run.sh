#!/bin/bash
# Counter passes (rocprofv3 --kernel-trace --pmc, one pass per run, nothing else traced) over one
# workload, then a markdown summary (tools/pmc_md.py).
# Usage (GPU box, repo root): bash tools/pmc_run.sh NAME [pmc_md args] -- python3 script.py args...
#   bash tools/pmc_run.sh gemm --labels gpurun_out/pmc_gemm_labels.json --match Cijk -- python3 tools/pmc_gemms.py --iters 4
#   bash tools/pmc_run.sh attn -- python3 tools/bench_attention.py --rounds 1 --iters 2
# -> gpurun_out/pmc_NAME/p{1,2}/ (raw csv), gpurun_out/pmc_NAME.md
# Slots per pass (MI355X_MICROARCH.md): <= 8 SQ, <= 4 TCC (FETCH_SIZE takes 3), <= 2 GRBM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD
NAME=$1; shift
MDARGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do MDARGS+=("$1"); shift; done
shift
CMD=()
for arg in "$@"; do if [ -e "$R/$arg" ]; then CMD+=("$R/$arg"); else CMD+=("$arg"); fi; done
PASSES=("SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
        "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE FETCH_SIZE")
# PMC_PASSES="A B C;D E F": custom passes (each within the per-block slot limits), raw means per kernel
# in gpurun_out/pmc_NAME.raw.md (tools/pmc_md.py --raw)
if [ -n "$PMC_PASSES" ]; then IFS=';' read -r -a PASSES <<< "$PMC_PASSES"; MDARGS+=("--raw"); fi
mkdir -p "gpurun_out/pmc_$NAME"
DIRS=()
i=0
for set in "${PASSES[@]}"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set --output-format csv \
     -d "$R/gpurun_out/pmc_$NAME/p$i" -o "$NAME" -- "${CMD[@]}" > "$R/gpurun_out/pmc_$NAME/p$i.log" 2>&1) \
    || { echo "pmc pass $i failed"; tail -5 "gpurun_out/pmc_$NAME/p$i.log"; exit 1; }
  DIRS+=("gpurun_out/pmc_$NAME/p$i")
done
python3 tools/pmc_md.py "${DIRS[@]}" "${MDARGS[@]}" --title "PMC: $NAME ($*)" > "gpurun_out/pmc_$NAME.md"
cat "gpurun_out/pmc_$NAME.md"
