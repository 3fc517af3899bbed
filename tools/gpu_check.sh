#!/bin/bash
# Round-end style check of the current tree on a GPU box (run through gpurun from the repo root):
# GPU test suite, smoke(), the driver's bench command, and a rocprofv3 kernel table of the headline step.
#   bash tools/gpu_check.sh OUT [suite|nosuite] [prof|noprof]
# -> gpurun_out/OUT/{pytest_gpu.log, smoke.log, bench.log, prof_lora.md}
# Every GPU step has its own time limit and the steps are chained: the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
OUT=gpurun_out/${1:-check}; SUITE=${2:-suite}; PROF=${3:-prof}
mkdir -p "$OUT"
if [ "$SUITE" = suite ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2>&1 \
  || { tail -20 "$OUT/bench.log"; exit 1; }
grep '^{' "$OUT/bench.log" | tail -1 | cut -c1-400
if [ "$PROF" = prof ]; then
  bash tools/prof_bench.sh lora_$1 --steps 3 --warmup 2 > /dev/null || exit 1
  cp gpurun_out/prof_lora_$1.md "$OUT/prof_lora.md"
  head -22 "$OUT/prof_lora.md"
fi
