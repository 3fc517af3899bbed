#!/bin/bash
# W64 vs 32-row flash forward: counters (one pass per run) + non-causal / shape timings -> gpurun_out/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_w64prof}; mkdir -p $O
timeout -k 10 120 python -u tools/bench_fwd_variants.py --noncausal > $O/fwd_ab_noncausal.log 2>&1 || exit 1
grep variant $O/fwd_ab_noncausal.log
timeout -k 10 120 python -u tools/bench_fwd_variants.py --B 16 --S 1024 > $O/fwd_ab_s1024.log 2>&1 || exit 1
grep variant $O/fwd_ab_s1024.log
bash tools/pmc_run.sh w64 -- python3 tools/bench_fwd_variants.py --rounds 1 --iters 2 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cp gpurun_out/pmc_w64.md $O/ && cat gpurun_out/pmc_w64.md
