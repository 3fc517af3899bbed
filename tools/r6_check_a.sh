set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/r6_a; mkdir -p $O
bash tools/gpu_check.sh r6_a suite noprof || exit 1
FTC_LAB=1 timeout -k 10 300 python -u -m pytest tests/test_gemm_lab.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lab.log 2>&1 || { tail -20 $O/pytest_lab.log; exit 1; }
tail -1 $O/pytest_lab.log
timeout -k 10 200 python -u tools/bench_attention.py --rounds 5 > $O/attn_base.log 2>&1 || { tail $O/attn_base.log; exit 1; }
cat $O/attn_base.log | tail -5
