#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6_w64diag; mkdir -p $O
timeout -k 10 120 python -u tools/diag_w64.py > $O/diag.log 2>&1; rc=$?; cat $O/diag.log | grep -v amdgpu.ids; exit $rc
