#!/bin/bash
# rocprofv3 kernel trace + stats of one bench.py configuration, summarised to markdown.
# Usage (GPU box, repo root): bash tools/prof_bench.sh NAME [bench.py args...]
#   bash tools/prof_bench.sh lora --steps 3 --warmup 2
#   bash tools/prof_bench.sh full --method full --steps 3 --warmup 2
# -> gpurun_out/prof_NAME/ (raw csv), gpurun_out/prof_NAME.md (per-step table), gpurun_out/prof_NAME.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD
NAME=$1; shift
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d "$R/gpurun_out/prof_$NAME" \
   -o "$NAME" -- python3 "$R/bench.py" "$@" > "$R/gpurun_out/prof_$NAME.log" 2>&1) || exit 1
python3 tools/kstats_md.py "gpurun_out/prof_$NAME" --log "gpurun_out/prof_$NAME.log" > "gpurun_out/prof_$NAME.md"
head -30 "gpurun_out/prof_$NAME.md"
