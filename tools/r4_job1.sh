set -o pipefail
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_nt or first_write" > gpurun_out/pytest_gemm.log 2>&1; tail -3 gpurun_out/pytest_gemm.log
OUT=rope_ab ARMS="lib=FTC_GEMM_NT=0 rope=FTC_GEMM_NT=rope all=FTC_GEMM_NT=1" ROUNDS=2 bash tools/step_ab.sh || exit 1
BACKEND=nccl REHEARSE_TIMEOUT=300 bash tools/rehearse_dp.sh 2 --model llama3-8b-1l --method full --steps 4 --warmup 2
