#!/bin/bash
# One gpurun session: GPU tests -> smoke -> short benches -> rocprofv3 kernel stats.
# Every GPU step has its own timeout; a crash/abort/timeout (rc >= 124 or signal) ends the session.
# Usage (from the repo root, on the GPU box): bash tools/gpu_session.sh [steps...]
#   steps: tests smoke bench1l bench bench_full bench_qlora bench_torch prof prof_lora prof_full attn ...
#   (default: tests smoke bench1l bench bench_torch prof)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
STEPS=("$@")
[ ${#STEPS[@]} -eq 0 ] && STEPS=(tests smoke bench1l bench bench_torch prof)

fatal() {  # rc -> 0 if the session may continue
  local rc=$1 name=$2
  echo "[session] $name rc=$rc"
  if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then
    echo "[session] $name crashed or timed out: stopping the session"
    exit "$rc"
  fi
  return 0
}

for s in "${STEPS[@]}"; do
  case "$s" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
      fatal $? tests; tail -5 gpurun_out/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      fatal $? smoke; tail -3 gpurun_out/smoke.log ;;
    bench1l)
      timeout -k 10 300 python bench.py --model llama3-8b-1l --steps 5 --warmup 2 > gpurun_out/bench1l.log 2>&1
      fatal $? bench1l; tail -2 gpurun_out/bench1l.log ;;
    bench)
      timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
      fatal $? bench; tail -2 gpurun_out/bench.log ;;
    attn)
      timeout -k 10 300 python tools/bench_attention.py > gpurun_out/bench_attn.log 2>&1
      fatal $? attn; tail -2 gpurun_out/bench_attn.log ;;
    attn_w8)
      FTC_FLASH_FWD_WAVES=8 timeout -k 10 300 python tools/bench_attention.py > gpurun_out/bench_attn_w8.log 2>&1
      fatal $? attn_w8; tail -2 gpurun_out/bench_attn_w8.log ;;
    flash_w8)
      FTC_FLASH_FWD_WAVES=8 timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or llama_lora" > gpurun_out/pytest_flash_w8.log 2>&1
      fatal $? flash_w8; tail -3 gpurun_out/pytest_flash_w8.log ;;
    attn_occ2)
      FTC_FLASH_BWD_OCC=2 timeout -k 10 300 python tools/bench_attention.py > gpurun_out/bench_attn_occ2.log 2>&1
      fatal $? attn_occ2; tail -2 gpurun_out/bench_attn_occ2.log ;;
    flash)
      timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k flash > gpurun_out/pytest_flash.log 2>&1
      fatal $? flash; tail -5 gpurun_out/pytest_flash.log ;;
    rccl2)  # 2 ranks on the ONE card through the bench launcher, RCCL over loopback sockets (NCCL_HOSTID per rank)
      FTC_SHARE_GPU=1 timeout -k 10 500 python bench.py --gpus 2 --model llama3-8b-1l --steps 5 --warmup 2 --comm-ab \
        --launcher-timeout 450 > gpurun_out/rccl2.log 2>&1
      fatal $? rccl2; grep '^{' gpurun_out/rccl2.log | cut -c1-2000 ;;
    rccl2_native)  # same, DDP buckets through the native engine (csrc/comm/rccl_engine.cpp)
      FTC_SHARE_GPU=1 timeout -k 10 500 python bench.py --gpus 2 --model llama3-8b-1l --steps 5 --warmup 2 \
        --comm-engine native --launcher-timeout 450 > gpurun_out/rccl2_native.log 2>&1
      fatal $? rccl2_native; grep '^{' gpurun_out/rccl2_native.log | cut -c1-2000 ;;
    rccl2_full)  # full FT, fp32 grads, ZeRO-1 reduce-scatter/all-gather over RCCL, 2 ranks on one card
      FTC_SHARE_GPU=1 timeout -k 10 500 python bench.py --gpus 2 --model llama3-8b-1l --method full --zero-stage 1 \
        --steps 4 --warmup 2 --comm-ab --launcher-timeout 450 > gpurun_out/rccl2_full.log 2>&1
      fatal $? rccl2_full; grep '^{' gpurun_out/rccl2_full.log | cut -c1-2000 ;;
    pipe_ab)  # flash forward in-wave software pipeline (FTC_FLASH_FWD_PIPE=1|2) -- numerics, then A/B
      for p in 1 2; do
        FTC_FLASH_FWD_PIPE=$p timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q \
          -k "flash or llama_lora or packed or tail or family" > gpurun_out/pytest_pipe$p.log 2>&1
        fatal $? pytest_pipe$p; tail -2 gpurun_out/pytest_pipe$p.log
      done
      for p in 0 1 2 0 1 2; do
        FTC_FLASH_FWD_PIPE=$p timeout -k 10 300 python tools/bench_attention.py --rounds 3 > gpurun_out/attn_pipe$p.log 2>&1
        fatal $? attn_pipe$p; grep -v amdgpu gpurun_out/attn_pipe$p.log | tail -1 | cut -c1-240
      done ;;
    conc_ab)  # flash backward: dQ on a side stream concurrent with dK/dV (FTC_FLASH_BWD_CONCURRENT) -- A/B
      timeout -k 10 300 python tools/bench_attention.py > gpurun_out/attn_conc0.log 2>&1
      fatal $? attn_conc0; grep -v amdgpu gpurun_out/attn_conc0.log | tail -3
      FTC_FLASH_BWD_CONCURRENT=1 timeout -k 10 300 python tools/bench_attention.py > gpurun_out/attn_conc1.log 2>&1
      fatal $? attn_conc1; grep -v amdgpu gpurun_out/attn_conc1.log | tail -3
      FTC_FLASH_BWD_CONCURRENT=1 timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or llama_lora or graph" \
        > gpurun_out/pytest_conc1.log 2>&1
      fatal $? pytest_conc1; tail -2 gpurun_out/pytest_conc1.log
      FTC_FLASH_BWD_CONCURRENT=1 timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_conc1.log 2>&1
      fatal $? bench_conc1; grep '^{' gpurun_out/bench_conc1.log | cut -c1-200
      timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_conc0.log 2>&1
      fatal $? bench_conc0; grep '^{' gpurun_out/bench_conc0.log | cut -c1-200 ;;
    sp2)  # Ulysses sequence parallelism, 2 ranks on the one card (RCCL over loopback): Llama-3-8B, 1 x 32k
      # tokens split 2 x 16k, heads <-> tokens all-to-all around full-sequence flash attention
      FTC_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --sp 2 --batch-size 1 --seq-len 32768 --steps 3 \
        --warmup 1 --launcher-timeout 550 > gpurun_out/sp2.log 2>&1
      fatal $? sp2; grep '^{' gpurun_out/sp2.log | cut -c1-900 ;;
    sp2_1l)  # same on the 1-layer model, 4 x 8k
      FTC_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --sp 2 --model llama3-8b-1l --batch-size 4 \
        --seq-len 8192 --steps 4 --warmup 2 --launcher-timeout 350 > gpurun_out/sp2_1l.log 2>&1
      fatal $? sp2_1l; grep '^{' gpurun_out/sp2_1l.log | cut -c1-900 ;;
    rccl4)  # 4 ranks on the one card (RCCL over loopback sockets), torch + native engines A/B, 1-layer
      FTC_SHARE_GPU=1 timeout -k 10 500 python bench.py --gpus 4 --model llama3-8b-1l --steps 4 --warmup 2 --comm-ab \
        --batch-size 2 --launcher-timeout 450 > gpurun_out/rccl4.log 2>&1
      fatal $? rccl4; grep '^{' gpurun_out/rccl4.log | cut -c1-2000 ;;
    bench_tail)  # seq_len not a multiple of the 256-row flash tile: tail-padded flash path vs 4096
      timeout -k 10 600 python bench.py --steps 6 --warmup 2 --seq-len 4000 > gpurun_out/bench_tail.log 2>&1
      fatal $? bench_tail; grep '^{' gpurun_out/bench_tail.log | cut -c1-400 ;;
    full_fp32)  # full FT, grad accumulation 2: fp32 vs bf16 gradient buffer (cost of the precise mode)
      timeout -k 10 600 python bench.py --method full --steps 4 --warmup 2 --grad-accum 2 --grad-dtype fp32 \
        > gpurun_out/full_fp32.log 2>&1
      fatal $? full_fp32; grep '^{' gpurun_out/full_fp32.log | cut -c1-600
      timeout -k 10 600 python bench.py --method full --steps 4 --warmup 2 --grad-accum 2 --grad-dtype bf16 \
        > gpurun_out/full_bf16.log 2>&1
      fatal $? full_bf16; grep '^{' gpurun_out/full_bf16.log | cut -c1-600 ;;
    tn)  # TN weight-gradient GEMM: numerics on both schedules, then the per-shape table (ours vs hipBLASLt)
      for s in 1 0; do
        FTC_GEMM_TN_SCHED=$s timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k gemm_tn \
          > gpurun_out/pytest_tn_sched$s.log 2>&1
        fatal $? pytest_tn_sched$s; tail -1 gpurun_out/pytest_tn_sched$s.log
      done
      for s in 1 0 1 0; do
        FTC_GEMM_TN_SCHED=$s timeout -k 10 300 python tools/bench_gemm_tn.py --cdtype bf16 > gpurun_out/bench_tn_sched$s.log 2>&1
        fatal $? bench_tn_sched$s; grep '^{' gpurun_out/bench_tn_sched$s.log | cut -c1-200
      done ;;
    full_tn)  # full FT step: weight gradients on hipBLASLt over transposed copies (0) vs the TN kernel (1)
      for t in 0 1 0 1; do
        FTC_GEMM_TN=$t timeout -k 10 400 python bench.py --method full --steps 6 --warmup 2 > gpurun_out/full_tn$t.log 2>&1
        fatal $? full_tn$t; grep '^{' gpurun_out/full_tn$t.log | cut -c80-150
      done ;;
    dw_side)  # full FT: weight gradients on a side stream (FTC_DW_STREAM=1) -- numerics, then interleaved A/B
      timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_distributed.py -m gpu -x -v \
        --timeout 200 --timeout-method thread -k "side_stream or rccl_matches_per_rank or overlapped" \
        > gpurun_out/pytest_dw_side.log 2>&1
      fatal $? pytest_dw_side; tail -3 gpurun_out/pytest_dw_side.log
      for t in 1a 0a 1b 0b; do
        FTC_DW_STREAM=${t:0:1} timeout -k 10 400 python bench.py --method full --steps 6 --warmup 2 > gpurun_out/full_dw$t.log 2>&1
        fatal $? full_dw$t; grep '^{' gpurun_out/full_dw$t.log | cut -c80-150
      done ;;
    prof_full_dw)  # kernel table of the side-stream full-FT step
      FTC_DW_STREAM=1 bash tools/prof_bench.sh full_dw --method full --steps 3 --warmup 2
      fatal $? prof_full_dw ;;
    qlora_aug)  # QLoRA: W / B / s A in one dequant launch (FTC_NF4_AUG=1) vs separate kernels -- numerics, A/B
      timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
        -k "nf4 or qlora" > gpurun_out/pytest_qlora_aug.log 2>&1
      fatal $? pytest_qlora_aug; tail -3 gpurun_out/pytest_qlora_aug.log
      for t in 1a 0a 1b 0b; do
        FTC_NF4_AUG=${t:0:1} timeout -k 10 400 python bench.py --model mistral-7b --method qlora --steps 8 --warmup 3 \
          > gpurun_out/qlora_aug$t.log 2>&1
        fatal $? qlora_aug$t; grep '^{' gpurun_out/qlora_aug$t.log | cut -c80-150
      done ;;
    hbm)  # per-kernel HBM read / write / TB/s of the 1-layer LoRA step, calibrated on a 1 GiB elementwise kernel
      PMC_PASSES="FETCH_SIZE GRBM_GUI_ACTIVE;WRITE_SIZE GRBM_GUI_ACTIVE" timeout -k 10 600 bash tools/pmc_run.sh hbm \
        -- python3 tools/hbm_probe.py > gpurun_out/hbm_run.log 2>&1
      fatal $? hbm
      python3 tools/pmc_md.py gpurun_out/pmc_hbm/p1 gpurun_out/pmc_hbm/p2 --hbm AUnaryFunctor \
        --title "HBM per kernel: 1-layer Llama-3-8B LoRA step" > gpurun_out/hbm_step.md 2>&1
      fatal $? hbm_md; head -30 gpurun_out/hbm_step.md ;;
    lora_wg)  # LoRA: adapter weight gradients on the side stream (FTC_LORA_WG_STREAM=1) -- numerics, headline A/B
      timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
        -k "side_stream" > gpurun_out/pytest_lora_wg.log 2>&1
      fatal $? pytest_lora_wg; tail -3 gpurun_out/pytest_lora_wg.log
      for t in 1a 0a 1b 0b; do
        FTC_LORA_WG_STREAM=${t:0:1} timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/lora_wg$t.log 2>&1
        fatal $? lora_wg$t; grep '^{' gpurun_out/lora_wg$t.log | cut -c80-150
      done ;;
    wgrad_wgs)  # swiglu_bwd_wgrad workgroup-count sweep (FTC_WGRAD_WGS: token-row blocks x column blocks)
      for w in 512 256 768 1024 1536 2048 512; do
        FTC_WGRAD_WGS=$w timeout -k 10 200 python tools/bench_swiglu_tail.py > gpurun_out/wgrad_wgs$w.log 2>&1
        fatal $? wgrad_wgs$w; echo "WGS=$w $(grep -E 'bwd_fused_wgrad|bwd_swiglu_only' gpurun_out/wgrad_wgs$w.log | tr '\n' ' ')"
      done ;;
    first_write)  # full FT: projection-weight gradients written by a beta = 0 first GEMM instead of zeroed -- A/B
      timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread \
        -k "first_write or side_stream" > gpurun_out/pytest_first_write.log 2>&1
      fatal $? pytest_first_write; tail -3 gpurun_out/pytest_first_write.log
      for t in 1a 0a 1b 0b; do
        FTC_GRAD_FIRST_WRITE=${t:0:1} timeout -k 10 400 python bench.py --method full --steps 6 --warmup 2 \
          > gpurun_out/first_write$t.log 2>&1
        fatal $? first_write$t; grep '^{' gpurun_out/first_write$t.log | cut -c80-150
      done ;;
    defaults_ab)  # headline LoRA step: this round's new defaults on vs off (side-stream dW, first-write gradients)
      for t in 1a 0a 1b 0b; do
        if [ "${t:0:1}" = 1 ]; then E="FTC_DW_STREAM=1 FTC_GRAD_FIRST_WRITE=1"; else E="FTC_DW_STREAM=0 FTC_GRAD_FIRST_WRITE=0"; fi
        env $E timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/defaults$t.log 2>&1
        fatal $? defaults$t; grep '^{' gpurun_out/defaults$t.log | cut -c80-150
      done ;;
    gemms)
      timeout -k 10 300 python tools/bench_gemms.py > gpurun_out/bench_gemms.log 2>&1
      fatal $? gemms; tail -3 gpurun_out/bench_gemms.log ;;
    bench_b8)
      timeout -k 10 600 python bench.py --steps 8 --warmup 3 --batch-size 8 > gpurun_out/bench_b8.log 2>&1
      fatal $? bench_b8; tail -2 gpurun_out/bench_b8.log ;;
    bench_full)
      timeout -k 10 600 python bench.py --method full --steps 6 --warmup 2 > gpurun_out/bench_full.log 2>&1
      fatal $? bench_full; tail -1 gpurun_out/bench_full.log | cut -c1-220 ;;
    bench_qlora)
      timeout -k 10 600 python bench.py --model mistral-7b --method qlora --steps 8 --warmup 3 > gpurun_out/bench_qlora.log 2>&1
      fatal $? bench_qlora; tail -1 gpurun_out/bench_qlora.log | cut -c1-220 ;;
    prof_lora)
      bash tools/prof_bench.sh lora --steps 3 --warmup 2
      fatal $? prof_lora ;;
    prof_full)
      bash tools/prof_bench.sh full --method full --steps 3 --warmup 2
      fatal $? prof_full ;;
    bench_torch)
      timeout -k 10 600 python bench.py --steps 10 --warmup 3 --kernels torch > gpurun_out/bench_torch.log 2>&1
      fatal $? bench_torch; tail -2 gpurun_out/bench_torch.log ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp)
      export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
        -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof.log 2>&1
      fatal $? prof; ls -R gpurun_out/prof | head -20 ;;
    gemm_shapes)  # plain timing of the step's hipBLASLt shapes (random operands)
      timeout -k 10 300 python tools/pmc_gemms.py --iters 10 > gpurun_out/gemm_shapes.log 2>&1
      fatal $? gemm_shapes; cat gpurun_out/gemm_shapes.log | grep '^{' ;;
    pmc_gemm)
      timeout -k 10 600 bash tools/pmc_run.sh gemm --labels gpurun_out/pmc_gemm_labels.json --match Cijk \
        -- python3 tools/pmc_gemms.py --iters 4 --labels "$PWD/gpurun_out/pmc_gemm_labels.json"
      fatal $? pmc_gemm ;;
    pmc_attn)
      timeout -k 10 600 bash tools/pmc_run.sh attn -- python3 tools/bench_attention.py --rounds 1 --iters 2
      fatal $? pmc_attn ;;
    pmc_step)  # every kernel of a 1-layer Llama-3-8B LoRA step (real shapes), grouped by kernel name
      timeout -k 10 600 bash tools/pmc_run.sh step -- python3 bench.py --model llama3-8b-1l --steps 2 --warmup 1
      fatal $? pmc_step ;;
    op_kernels)  # kernel -> launching op attribution, 1-layer LoRA step (torch.profiler)
      timeout -k 10 300 python tools/op_kernels.py --top 60 > gpurun_out/op_kernels.md 2> gpurun_out/op_kernels.err
      fatal $? op_kernels; head -30 gpurun_out/op_kernels.md ;;
    pp2_ab)  # dK/dV half-1 order B1 B2 A (FTC_FLASH_DKDV_PP2) -- stamps, numerics, interleaved A/B, bench
      FTC_FLASH_DKDV_PP2=1 timeout -k 10 120 ./tools/stamp_dkdv 0 256 > gpurun_out/stamp_dkdv_pp2.md 2>&1
      fatal $? stamp_pp2; head -12 gpurun_out/stamp_dkdv_pp2.md
      FTC_FLASH_DKDV_PP2=1 timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q \
        -k "flash or llama_lora or packed or tail or family" > gpurun_out/pytest_pp2.log 2>&1
      fatal $? pytest_pp2; tail -2 gpurun_out/pytest_pp2.log
      for p in 0 1 0 1; do
        FTC_FLASH_DKDV_PP2=$p timeout -k 10 300 python tools/bench_attention.py --rounds 3 > gpurun_out/attn_pp2_$p.log 2>&1
        fatal $? attn_pp2_$p; grep -v amdgpu gpurun_out/attn_pp2_$p.log | tail -1 | cut -c1-300
      done
      FTC_FLASH_DKDV_PP2=1 timeout -k 10 600 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_pp2.log 2>&1
      fatal $? bench_pp2; grep '^{' gpurun_out/bench_pp2.log | cut -c1-200 ;;
    *) echo "unknown step $s" ;;
  esac
done
echo "[session] done"
