#!/usr/bin/env python3
"""Interleaved timing of the lab builds (tools/w64_lab/lib*.so) at the Llama-3-8B layer shape; the abl_*
builds are timing-only ablations (their outputs are wrong by construction)."""
import ctypes
import glob
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from diag import load  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    libs = {os.path.basename(p)[3:-3]: load(p) for p in sorted(glob.glob(os.path.join(HERE, "lib*.so")))}
    B, S, H, KV, D = 4, 4096, 32, 8, 128
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (H + 2 * KV) * D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + KV) * D], qkv[:, (H + KV) * D:]
    o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    arms = [(n, 1) for n in libs if n != "w32pin"] + [("base", 2), ("base", 0)] + \
        ([("w32pin", 0)] if "w32pin" in libs else [])
    times = {f"{n}/{v}": [] for n, v in arms}

    def call(L):
        return L.ftc_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, H, KV, D,
                               q.stride(0), k.stride(0), o.stride(0), 1 / math.sqrt(D), 1, 0, None, S, st)
    for n, var in arms:
        libs[n].ftc_flash_fwd_config(var)
        assert call(libs[n]) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(7):
        for n, var in arms:
            L = libs[n]
            L.ftc_flash_fwd_config(var)
            e0.record()
            for _ in range(20):
                call(L)
            e1.record()
            torch.cuda.synchronize()
            times[f"{n}/{var}"].append(e0.elapsed_time(e1) / 20)
    for kname, t in times.items():
        print(json.dumps({"arm": kname.replace("/1", " (persistent)").replace("/2", " (per-block)").replace("/0", " (w32)"), "ms_median": round(sorted(t)[3], 4)}))


if __name__ == "__main__":
    main()
