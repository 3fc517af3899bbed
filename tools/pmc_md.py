#!/usr/bin/env python3
"""Summarise rocprofv3 ``--pmc`` passes (one directory per pass) as a markdown table.

    python tools/pmc_md.py gpurun_out/pmc_gemm/p1 gpurun_out/pmc_gemm/p2 [--labels shapes.json]
        [--match Cijk] [--title ...]

Per kernel (or per labelled GEMM shape, see tools/pmc_gemms.py) it reports the mean dispatch time
(kernel trace), the effective clock ``GRBM_GUI_ACTIVE / 8 / time`` (the counter is summed over the 8
XCDs; MI355X_MICROARCH.md 'DVFS give-back'), the matrix-pipe busy share
``SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 1024 SIMDs)``, the stall split of the wave cycles
(``SQ_WAIT_INST_ANY`` issue stalls, ``SQ_WAIT_ANY`` parked on waitcnt/barrier), LDS bank-conflict
cycles per LDS-array cycle, and HBM fetch (``FETCH_SIZE`` x 2: gfx950 tallies 128-B requests at 64 B).
For labelled shapes with known FLOPs it adds achieved TFLOP/s and the FLOPs per clock as a share of
the 1024 FLOP/clk/SIMD bf16 MFMA rate (clock-independent utilisation).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

SIMDS = 256 * 4
BF16_FLOP_PER_CLK_SIMD = 1024


def _col(row, *names):
    low = {k.lower(): k for k in row}
    for n in names:
        if n.lower() in low:
            return row[low[n.lower()]]
    return None


def load_pass(d):
    """{dispatch_id: {"name", "counters": {..}, "ns"}} for one pass directory."""
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(_col(r, "Dispatch_Id", "Correlation_Id"))
            e = out.setdefault(did, {"name": _col(r, "Kernel_Name"), "counters": {}, "ns": None})
            cname, cval = _col(r, "Counter_Name"), _col(r, "Counter_Value")
            if cname is not None and cval not in (None, ""):
                e["counters"][cname] = e["counters"].get(cname, 0.0) + float(cval)
            st, en = _col(r, "Start_Timestamp"), _col(r, "End_Timestamp")
            if st and en and int(en) > int(st):
                e["ns"] = int(en) - int(st)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            did = int(_col(r, "Dispatch_Id", "Correlation_Id"))
            if did in out:
                out[did]["ns"] = int(_col(r, "End_Timestamp")) - int(_col(r, "Start_Timestamp"))
                out[did]["name"] = out[did]["name"] or _col(r, "Kernel_Name")
    return out


def _short(name: str) -> str:
    """Kernel name without namespaces, return type and argument list (templates kept)."""
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    depth = 0
    for i, ch in enumerate(n):
        depth += ch == "<"
        depth -= ch == ">"
        if ch == "(" and depth == 0:
            n = n[:i]
            break
    return n[:100]


def group(disp, labels, match):
    """Aggregate dispatches per key: the labelled shape (sentinel-split) or the kernel name."""
    agg = defaultdict(lambda: {"n": 0, "ns": 0.0, "c": defaultdict(float)})
    cur = -1
    shapes = labels["shapes"] if labels else None
    for did in sorted(disp):
        e = disp[did]
        name = e["name"] or "?"
        if shapes is not None and "FillFunctor<unsigned char>" in name:
            cur += 1
            continue
        if match and not any(m in name for m in match.split(",")):
            continue
        if shapes is not None:
            if cur < 0 or cur >= len(shapes):
                continue
            key = shapes[cur]["label"] + (" [ours]" if "gemm_nt" in name else "")
        else:
            key = _short(name)
        a = agg[key]
        a["n"] += 1
        a["ns"] += e["ns"] or 0.0
        for k, v in e["counters"].items():
            a["c"][k] += v
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--labels", default=None)
    ap.add_argument("--match", default=None, help="only kernels whose name contains this (comma: any of)")
    ap.add_argument("--title", default="rocprofv3 PMC summary")
    ap.add_argument("--raw", action="store_true", help="every counter's mean per dispatch (custom passes)")
    ap.add_argument("--hbm", default=None, metavar="CALIB_MATCH",
                    help="per-kernel HBM read / write GB and TB/s from FETCH_SIZE + WRITE_SIZE, scaled by the "
                         "kernel whose name contains CALIB_MATCH (1 GiB read + 1 GiB written per dispatch)")
    a = ap.parse_args()
    labels = json.load(open(a.labels)) if a.labels else None
    merged = {}
    for d in a.dirs:
        for key, v in group(load_pass(d), labels, a.match).items():
            m = merged.setdefault(key, {"n": v["n"], "ns": v["ns"], "c": {}})
            m["n"], m["ns"] = max(m["n"], v["n"]), max(m["ns"], v["ns"])  # time: same kernel every pass
            for k, x in v["c"].items():
                m["c"].setdefault(k, x / max(v["n"], 1))
    flops = {s["label"]: s for s in labels["shapes"]} if labels else {}
    print(f"# {a.title}\n")
    if a.hbm:
        return hbm_table(merged, a.hbm)
    if a.raw:  # per kernel: us, clock, then every counter as a mean per dispatch (cycles counters also / wave cycles)
        names = sorted({k for m in merged.values() for k in m["c"]})
        print("| kernel | disp | us | clock GHz | " + " | ".join(names) + " |")
        print("|" + "---|" * (4 + len(names)))
        for key, m in sorted(merged.items(), key=lambda kv: -kv[1]["ns"] / max(kv[1]["n"], 1)):
            us = m["ns"] / max(m["n"], 1) / 1e3
            gui = m["c"].get("GRBM_GUI_ACTIVE")
            clk = f"{gui / 8 / (us * 1e3):.2f}" if gui and us else ""
            vals = " | ".join(f"{m['c'][k]:.4g}" if k in m["c"] else "" for k in names)
            print(f"| `{key}` | {m['n']} | {us:.1f} | {clk} | {vals} |")
        return
    hdr = ("| kernel / shape | disp | us | clock GHz | MFMA busy | FLOP/clk share | TF/s | WAIT_INST_ANY | WAIT_ANY |"
           " LDS confl/active | HBM GB |")
    print(hdr + "\n|" + "---|" * (hdr.count("|") - 1))
    for key, m in sorted(merged.items(), key=lambda kv: -kv[1]["ns"] / max(kv[1]["n"], 1)):
        c = m["c"]
        us = m["ns"] / max(m["n"], 1) / 1e3
        gui = c.get("GRBM_GUI_ACTIVE")
        clk = gui / 8 / (us * 1e3) if gui and us else None
        cyc = gui / 8 if gui else None
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        busy = mf / (cyc * SIMDS) if mf is not None and cyc else None
        wc = c.get("SQ_WAVE_CYCLES")
        wia = c.get("SQ_WAIT_INST_ANY") / wc if wc and "SQ_WAIT_INST_ANY" in c else None
        wa = c.get("SQ_WAIT_ANY") / wc if wc and "SQ_WAIT_ANY" in c else None
        lds = (c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
               if c.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in c else None)
        hbm = 2 * c["FETCH_SIZE"] / 1e6 if "FETCH_SIZE" in c else None  # FETCH_SIZE is in KB
        tf = share = None
        fk = key.replace(" [ours]", "")
        if fk in flops and us:
            tf = flops[fk]["flops"] / (us * 1e-6) / 1e12
            if cyc:
                share = flops[fk]["flops"] / (cyc * SIMDS * BF16_FLOP_PER_CLK_SIMD)

        def f(v, p=3):
            return "" if v is None else f"{v:.{p}f}"
        print(f"| `{key}` | {m['n']} | {us:.1f} | {f(clk, 2)} | {f(busy)} | {f(share)} | {f(tf, 0)} | {f(wia)} | "
              f"{f(wa)} | {f(lds)} | {f(hbm, 2)} |")


def hbm_table(merged, calib_match):
    """Achieved HBM bandwidth per kernel: counts scaled so the calibration kernel reads and writes 1 GiB."""
    cal = [m for k, m in merged.items() if calib_match in k]
    if not cal or "FETCH_SIZE" not in cal[0]["c"] or "WRITE_SIZE" not in cal[0]["c"]:
        raise SystemExit(f"no calibration kernel matching {calib_match!r} with FETCH_SIZE and WRITE_SIZE")
    gib = float(1 << 30)
    rs, ws = gib / cal[0]["c"]["FETCH_SIZE"], gib / cal[0]["c"]["WRITE_SIZE"]
    cus = cal[0]["ns"] / max(cal[0]["n"], 1) / 1e3
    print(f"calibration `{calib_match}`: {cus:.1f} us per 1 GiB read + 1 GiB written = "
          f"{2 * gib / (cus * 1e-6) / 1e12:.2f} TB/s; bytes per FETCH_SIZE count {rs:.1f}, per WRITE_SIZE count "
          f"{ws:.1f}\n")
    print("| kernel | disp | us | read GB | write GB | TB/s |\n|---|---|---|---|---|---|")
    rows = []
    for key, m in merged.items():
        c = m["c"]
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c or calib_match in key:
            continue
        us = m["ns"] / max(m["n"], 1) / 1e3
        rd, wr = c["FETCH_SIZE"] * rs / 1e9, c["WRITE_SIZE"] * ws / 1e9
        rows.append((us * m["n"], key, m["n"], us, rd, wr, (rd + wr) / (us * 1e-6) / 1e3 if us else 0.0))
    for _, key, n, us, rd, wr, tbs in sorted(rows, reverse=True):
        print(f"| `{key}` | {n} | {us:.1f} | {rd:.3f} | {wr:.3f} | {tbs:.2f} |")


if __name__ == "__main__":
    main()
