mkdir -p gpurun_out/gemm_r4 && timeout -k 10 300 python -u tools/bench_gemm_nt.py --shapes qkv_fwd,gu_fwd,down_dx,down_fwd --configs "$CFG" > gpurun_out/gemm_r4/$LOG 2>&1
python3 tools/gemm_sweep_summary.py gpurun_out/gemm_r4/$LOG
