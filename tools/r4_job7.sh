#!/bin/bash
# IL dK/dV vs 8-wave: per-kernel times (rocprofv3 --stats) and counters; full-FT step with split-K dW (down) A/B
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/attn_r4 gpurun_out/dw_r4
R=$PWD
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/attn_r4/stats_bwd -o bwd -- python3 $R/tools/bench_attn_bwd.py --rounds 2 --iters 5 > $R/gpurun_out/attn_r4/stats_bwd.log 2>&1); rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/attn_r4/stats_bwd.log; exit $rc; }
f=$(find gpurun_out/attn_r4/stats_bwd -name "*kernel_stats.csv" | head -1); python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'dkdv' in r['Name'] or 'dq' in r['Name'] or 'delta' in r['Name']: print(r['Name'][:70], r['Calls'], r['AverageNs'])"
bash tools/pmc_run.sh bwdil -- python3 tools/bench_attn_bwd.py --rounds 1 --iters 2 > gpurun_out/attn_r4/pmc_bwdil.log 2>&1; rc=$?; tail -30 gpurun_out/attn_r4/pmc_bwdil.log | grep -i "dkdv\|kernel\|---" ; [ $rc -eq 0 ] || exit $rc
OUT=dw_r4/full_ab ROUNDS=2 STEPS=6 WARMUP=2 BENCH_ARGS="--method full" ARMS="base=FTC_DW_SPLIT=0 split=FTC_DW_SPLIT=auto" bash tools/step_ab.sh
