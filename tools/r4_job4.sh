#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/gemm_r4
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_nt" > gpurun_out/gemm_r4/pytest_m0walk.log 2>&1; rc=$?; tail -2 gpurun_out/gemm_r4/pytest_m0walk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_gemm_nt.py --shapes qkv_fwd,o_fwd,gu_fwd,down_dx,down_fwd,gu_dx --configs "0,-8,32,0;0,8,32,0;100000,-8,32,0" > gpurun_out/gemm_r4/m0walk.log 2>&1; rc=$?; python3 tools/gemm_sweep_summary.py gpurun_out/gemm_r4/m0walk.log; exit $rc
