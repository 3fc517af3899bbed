#!/bin/bash
# Round 6: the lab W64 flash forward on one GPU -> gpurun_out/<out>/ (numerics first; timing only if they pass).
# Needs the lab build: bash tools/w64_lab/build.sh (here, before the gpurun call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6_w64}; mkdir -p $O
timeout -k 10 120 python -u tools/w64_lab/diag.py > $O/lab_diag.log 2>&1 || { tail -20 $O/lab_diag.log; exit 1; }
grep -v amdgpu.ids $O/lab_diag.log
FTC_LAB=1 timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_w64_lab.py \
  > $O/pytest.log 2>&1 || { grep -E "^E|FAILED|Error" $O/pytest.log | head -30; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2; grep "^w64" $O/pytest.log | head -20
timeout -k 10 180 python -u tools/w64_lab/timing.py > $O/timing.log 2>&1 || { tail $O/timing.log; exit 1; }
grep arm $O/timing.log
