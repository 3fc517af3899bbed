#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--stats`` kernel_stats.csv as a per-step markdown table.

The number of profiled steps is steps + warmup read from the bench JSON line in ``--log`` (every
step, warm-up included, runs under the profiler)."""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--log", default=None)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_stats.csv under {a.dir}")
    steps, line = 1, None
    if a.log and os.path.exists(a.log):
        for ln in open(a.log):
            if ln.startswith("{") and '"metric"' in ln:
                line = json.loads(ln)
        if line:
            steps = int(line["steps"]) + int(line["warmup"])
    rows = list(csv.DictReader(open(files[0])))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# rocprofv3 kernel stats: `bench.py` {json.dumps(line['config']) if line else ''}\n")
    if line:
        print(f"bench line under the profiler: {line['value']:.0f} {line['unit']}, {line['ms_per_step']:.1f} ms/step; "
              f"{steps} profiled steps (warm-up included), per-step = total / {steps}.\n")
    print("| ms/step | calls/step | avg us | % | kernel |\n|---:|---:|---:|---:|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        t = float(r["TotalDurationNs"])
        print(f"| {t / 1e6 / steps:.2f} | {int(r['Calls']) / steps:.1f} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"{100 * t / tot:.1f} | `{r['Name'][:110]}` |")
    print(f"| **{tot / 1e6 / steps:.1f}** | | | | total GPU kernel time per step |")


if __name__ == "__main__":
    main()
