#!/bin/bash
# rocprofv3 kernel-trace + stats of the attention microbenchmark and of the flagship bench.
# Usage (GPU box, repo root): bash tools/prof_session.sh [attn] [bench]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in "$@"; do
  case "$s" in
    attn)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_attn -o attn \
        -- python3 tools/bench_attention.py --rounds 1 > gpurun_out/prof_attn.log 2>&1 || exit $? ;;
    bench)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench \
        -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof.log 2>&1 || exit $? ;;
  esac
done
find gpurun_out/prof* -name "*kernel_stats.csv" | head
