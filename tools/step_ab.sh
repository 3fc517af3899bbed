#!/bin/bash
# Interleaved A/B of the headline step under environment settings: ARMS="NAME=ENV ..." (env assignments
# joined by commas), ROUNDS rounds; logs + one summary line per run under gpurun_out/$OUT/.
set -o pipefail
out=gpurun_out/${OUT:-step_ab}; mkdir -p $out
for r in $(seq 1 ${ROUNDS:-2}); do
  for arm in $ARMS; do
    name=${arm%%=*}; envs=${arm#*=}
    env $(echo $envs | tr ',' ' ') timeout -k 10 ${STEP_TIMEOUT:-300} python -u bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} $BENCH_ARGS > $out/${name}_r$r.log 2>&1 || { echo "FAILED $name r$r"; tail -20 $out/${name}_r$r.log; exit 1; }
    echo "$name r$r $(grep '^{' $out/${name}_r$r.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
