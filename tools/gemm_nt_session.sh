#!/bin/bash
# One GPU call: numerics of the hand-written projection GEMM (+ the attention / parity tests touched this
# round), the per-shape table against hipBLASLt for the default variant and an older one, and a counter
# pass of the default variant.  Usage (GPU box, repo root): bash tools/gemm_nt_session.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/gemm_nt}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "gemm_nt or flash_tail or fp32_model or flash_attention_fwd_bwd" > "$OUT/pytest.log" 2>&1
echo "pytest rc=$?" >> "$OUT/pytest.log"
timeout -k 10 300 python -u tools/bench_gemm_nt.py --iters 10 --rounds 2 > "$OUT/bench_default.log" 2>&1 || exit 1
FTC_GEMM_NT_VARIANT=1 timeout -k 10 200 python -u tools/bench_gemm_nt.py --shapes gu_fwd,down_dx,qkv_fwd --iters 10 \
  --rounds 2 > "$OUT/bench_v1.log" 2>&1 || exit 1
PMC_PASSES="SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCC_HIT TCC_MISS" \
  timeout -k 10 300 bash tools/pmc_run.sh ntv5 -- python3 tools/bench_gemm_nt.py --shapes gu_fwd --iters 3 --rounds 1 > /dev/null
cp gpurun_out/pmc_ntv5.md "$OUT/" 2>/dev/null
exit 0
