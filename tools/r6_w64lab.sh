#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_w64lab; mkdir -p $O
timeout -k 10 120 python -u tools/w64_lab/${1:-diag}.py > $O/${1:-diag}.log 2>&1; rc=$?; grep -v amdgpu.ids $O/${1:-diag}.log; exit $rc
