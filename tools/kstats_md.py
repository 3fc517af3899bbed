#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--stats`` kernel_stats.csv as a per-step markdown table.

With a marker trace (``rocprofv3 --marker-trace``) holding bench.py's ``ftc_timed`` roctx range, only
the kernels that START inside the timed region are counted and divided by the timed step count (no
initialisation / warm-up kernels).  Otherwise the whole ``kernel_stats.csv`` is divided by steps +
warmup read from the bench JSON line in ``--log`` (every step, warm-up included, ran under the
profiler)."""
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
    timed = _timed_rows(a.dir)
    if timed is not None and line:
        rows, steps = timed, int(line["steps"])
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# rocprofv3 kernel stats: `bench.py` {json.dumps(line['config']) if line else ''}\n")
    if line:
        what = (f"{steps} timed steps (kernels inside the `ftc_timed` roctx range only)" if timed is not None else
                f"{steps} profiled steps (warm-up and initialisation included)")
        print(f"bench line under the profiler: {line['value']:.0f} {line['unit']}, {line['ms_per_step']:.1f} ms/step; "
              f"{what}, per-step = total / {steps}.\n")
    print("| ms/step | calls/step | avg us | % | kernel |\n|---:|---:|---:|---:|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
        t = float(r["TotalDurationNs"])
        print(f"| {t / 1e6 / steps:.2f} | {int(r['Calls']) / steps:.1f} | {float(r['AverageNs']) / 1e3:.1f} | "
              f"{100 * t / tot:.1f} | `{r['Name'][:110]}` |")
    print(f"| **{tot / 1e6 / steps:.1f}** | | | | total GPU kernel time per step |")


def _timed_rows(d):
    """Per-kernel aggregates over the kernels that start inside the ftc_timed marker range, or None."""
    marks = glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True)
    traces = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not marks or not traces:
        return None
    lo = hi = None
    for r in csv.DictReader(open(marks[0])):
        if any("ftc_timed" in str(v) for v in r.values()):  # message column name varies by version
            lo, hi = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if lo is None:
        return None
    agg: dict[str, list] = {}
    for r in csv.DictReader(open(traces[0])):
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if lo <= st <= hi:
            e = agg.setdefault(r["Kernel_Name"], [0, 0.0])
            e[0] += 1
            e[1] += en - st
    return [{"Name": k, "Calls": c, "TotalDurationNs": t, "AverageNs": t / c} for k, (c, t) in agg.items()]


if __name__ == "__main__":
    main()
