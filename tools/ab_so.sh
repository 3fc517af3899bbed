#!/bin/bash
# A/B builds of the kernel extension on one box: finetune_controller_amd/_C_a.so, _C_b.so, ... (VARIANTS,
# default "a b"; built here beforehand) are copied in turn over _C.so and the same command runs against each, alternating
# for ROUNDS rounds (box drift hits both arms).  Usage (from gpurun):
#   ROUNDS=3 OUT=name bash tools/ab_so.sh 'python -u tools/bench_attention.py' 'python -u bench.py'
# -> gpurun_out/OUT/{a,b}_<cmd index>_r<round>.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/${OUT:-ab_so}; mkdir -p $O
P=finetune_controller_amd
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-a b}; do
    cp $P/_C_$v.so $P/_C.so || exit 1
    i=0
    for c in "$@"; do
      i=$((i + 1))
      timeout -k 10 ${STEP_TIMEOUT:-300} $c > $O/${v}_${i}_r$r.log 2>&1 || { tail -20 $O/${v}_${i}_r$r.log; exit 1; }
      echo "$v cmd$i r$r: $(grep -h '^{' $O/${v}_${i}_r$r.log | tail -1 | cut -c1-${CUT:-330})"
    done
  done
done
