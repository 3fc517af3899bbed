#!/usr/bin/env python3
"""Structured-input probes of the W64 forward's wrong rows (tools/w64_lab/libbase.so)."""
import ctypes
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from diag import load, ref  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def fwd(L, q, k, v, B, S, H, KV, D, causal):
    o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
    rc = L.ftc_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, H, KV, D,
                         q.stride(0), k.stride(0), o.stride(0), 1 / math.sqrt(D), int(causal), 0, None, S,
                         ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert rc == 0
    return o.float()


def main():
    L = load(os.path.join(HERE, "libbase.so"))
    L.ftc_flash_fwd_config(1)
    B, S, H, KV, D = 1, 256, 1, 1, 128
    torch.manual_seed(0)
    # (b) one-hot V: O[q][d] = P[q][d] + P[q][d + 128]
    q = torch.randn(S, D, device="cuda").bfloat16()
    k = torch.randn(S, D, device="cuda").bfloat16()
    v = torch.zeros(S, D, device="cuda")
    v[torch.arange(S), torch.arange(S) % D] = 1.0
    v = v.bfloat16()
    for causal in (False, True):
        o = fwd(L, q, k, v, B, S, H, KV, D, causal)
        r = ref(q, k, v, B, S, H, KV, D, causal)
        d = (o - r).abs()
        bad_rows = (d.amax(-1) > 2e-3).nonzero().flatten().tolist()
        print(f"one-hot V causal={causal}: bad rows {len(bad_rows)}: {bad_rows[:40]}")
        for row in bad_rows[:4]:
            cols = (d[row] > 2e-3).nonzero().flatten().tolist()
            print(f"  row {row} (wave {row // 64} j {(row % 64) // 32} lr {row % 32}): bad d {cols[:40]}")
            print("    ours", [round(x, 4) for x in o[row, cols[:8]].tolist()], " ref", [round(x, 4) for x in r[row, cols[:8]].tolist()])
    # (a) identical Q rows: every O row equal
    q1 = q[:1].repeat(S, 1).contiguous()
    v2 = torch.randn(S, D, device="cuda").bfloat16()
    o = fwd(L, q1, k, v2, B, S, H, KV, D, False)
    dd = (o - o[:1]).abs().amax(-1)
    print("identical-Q rows differing from row 0:", (dd > 1e-3).nonzero().flatten().tolist()[:40])


if __name__ == "__main__":
    main()
