#!/bin/bash
# gemm_nt: M0-walk DMA + operand cache-policy variants -- tests, then an interleaved sweep
set -o pipefail
mkdir -p gpurun_out/gemm_r4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_nt" > gpurun_out/gemm_r4/pytest_m0walk.log 2>&1; rc=$?; tail -2 gpurun_out/gemm_r4/pytest_m0walk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_gemm_nt.py --rounds 4 --shapes qkv_fwd,o_fwd,gu_fwd,down_dx,down_fwd --configs "0,-8,32,0,0;0,-8,32,0,1;0,-8,32,0,2;0,-8,32,0,3;0,-8,32,0,4" > gpurun_out/gemm_r4/policy.log 2>&1; rc=$?; python3 tools/gemm_sweep_summary.py gpurun_out/gemm_r4/policy.log; exit $rc
