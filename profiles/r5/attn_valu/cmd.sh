#!/bin/bash
# Attention kernels' instruction mix: transcendental (v_exp) vs FMA / MUL / ADD VALU vs MFMA issue, and
# the VALU-MFMA co-execution share (VERDICT r4 "Next" 2: the softmax's exp share).  The counter names are
# checked against `rocprofv3 --list-avail` first; one pass per run.  -> gpurun_out/pmc_attn_valu.raw.md
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$PWD
(cd /tmp && timeout -k 10 120 rocprofv3 --list-avail > "$R/gpurun_out/avail.txt" 2>&1) || true
have() { grep -q -w "$1" gpurun_out/avail.txt; }
p1=""; for c in SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_INSTS_MFMA SQ_INSTS_LDS; do have $c && p1="$p1 $c"; done
p2=""; for c in SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE; do have $c && p2="$p2 $c"; done
echo "pass1:$p1"; echo "pass2:$p2"
PMC_PASSES="${p1# };${p2# }" bash tools/pmc_run.sh attn_valu -- python3 tools/bench_attention.py --rounds 1 --iters 2
