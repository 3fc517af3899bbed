#!/bin/bash
# round-4 projection GEMM session: correctness (persistent multi-tile + production shapes), then the
# launch-configuration sweep against hipBLASLt (tools/bench_gemm_nt.py), logs under gpurun_out/gemm_r4/
set -o pipefail
out=gpurun_out/gemm_r4; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm_nt" > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
CFG=${CFG:-"0,8,32,0;0,16,2,0;0,16,2,1;0,8,32,1;100000,8,32,0;0,4,32,0;0,-8,32,0;0,8,8,0"}
timeout -k 10 400 python -u tools/bench_gemm_nt.py --shapes ${SHAPES:-qkv_fwd,o_fwd,gu_fwd,down_dx,down_fwd} --configs "$CFG" > $out/sweep.log 2>&1 || { tail -20 $out/sweep.log; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/gemm_r4/sweep.log"):
    if l.startswith("{"):
        d=json.loads(l); print(d["gemm"], d["config"], d["ours_tf"], d["lib_tf"], d["speedup"], d["max_rel_err_vs_lib"])
PY
