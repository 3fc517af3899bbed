#!/bin/bash
# Flash forward row-max exchange A/B: v_permlane32_swap (default) vs ds_bpermute (FTC_FLASH_FWD_XHALF=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "flash or llama_lora or packed or tail" \
  > gpurun_out/pytest_xhalf.log 2>&1 || { tail -5 gpurun_out/pytest_xhalf.log; exit 1; }
tail -1 gpurun_out/pytest_xhalf.log
for x in 1 0 1 0; do
  FTC_FLASH_FWD_XHALF=$x timeout -k 10 300 python tools/bench_attention.py --rounds 3 > gpurun_out/attn_xhalf$x.log 2>&1 || exit 1
  echo "xhalf=$x $(grep -v amdgpu gpurun_out/attn_xhalf$x.log | tail -1 | cut -c1-200)"
done
for x in 1 0; do
  FTC_FLASH_FWD_XHALF=$x timeout -k 10 400 python bench.py --steps 8 --warmup 2 > gpurun_out/bench_xhalf$x.log 2>&1 || exit 1
  echo "bench xhalf=$x $(grep '^{' gpurun_out/bench_xhalf$x.log | cut -c80-140)"
done
