#!/bin/bash
# Round 6: counter passes over the W64 forward (persistent, per-block) and the 32-row kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in 1 2 0; do
  bash tools/pmc_run.sh w64v$v -- python3 tools/w64_lab/one.py base $v 3 > /dev/null || exit 1
done
for v in 1 2 0; do echo "== variant $v"; grep -v "^$" gpurun_out/pmc_w64v$v.md | tail -8; done
