#!/bin/bash
# Round 6: W64 numerics + forward A/B (tools/r6_w64.sh), then the lab ablation timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r6_w64.sh ${1:-r6_w64f} && bash tools/r6_w64lab.sh timing
