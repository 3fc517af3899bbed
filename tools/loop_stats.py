#!/usr/bin/env python3
"""Instruction mix of every backward-branch loop of one kernel in a hipcc ``-S`` listing.

    python tools/loop_stats.py out.s flash_fwd_w64_kernel

Prints, per loop (label, instruction count): MFMAs, SGPR spill lane moves, scratch ops, waits, nops,
LDS reads and exponentials -- the first thing to read after a schedule change.
"""
import re
import sys


def main(path: str, kernel: str) -> None:
    L = open(path).read().split("\n")
    st = next(i for i, l in enumerate(L) if kernel in l and re.match(r"^_Z\S*:", l))
    en = next(i for i in range(st, len(L)) if L[i].strip().startswith("s_endpgm"))
    body = L[st:en]
    labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    keys = ["v_mfma", "v_readlane", "v_writelane", "scratch_", "s_waitcnt", "s_nop", "ds_read", "v_exp", "s_barrier"]
    for i, l in enumerate(body):
        m = re.search(r"s_c?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            seg = [x.strip() for x in body[labels[m.group(1)]:i] if x.strip() and not x.strip().startswith((".", ";"))]
            print(m.group(1), len(seg), " ".join(f"{k.strip('_')}={sum(1 for x in seg if x.startswith(k))}" for k in keys))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
