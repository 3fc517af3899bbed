#!/bin/bash
# rocprofv3 kernel stats of the generation benchmark (tools/bench_decode.py args pass through).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_decode" \
   -o decode -- python3 "$R/tools/bench_decode.py" "$@" > "$R/gpurun_out/prof_decode.log" 2>&1) || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_decode/**/decode_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel ms {tot/1e6:.1f}")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):7d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
