#!/usr/bin/env python3
"""Run one lab build / variant of the flash forward a few times at the Llama-3-8B layer shape (for counter
passes): python tools/w64_lab/one.py base 1 [iters]"""
import ctypes
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from diag import load  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    name, var = sys.argv[1], int(sys.argv[2])
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    L = load(os.path.join(HERE, f"lib{name}.so"))
    L.ftc_flash_fwd_config(var)
    B, S, H, KV, D = 4, 4096, 32, 8, 128
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (H + 2 * KV) * D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + KV) * D], qkv[:, (H + KV) * D:]
    o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(iters):
        assert L.ftc_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, H, KV, D,
                               q.stride(0), k.stride(0), o.stride(0), 1 / math.sqrt(D), 1, 0, None, S, st) == 0
    torch.cuda.synchronize()
    print("ok", name, var)


if __name__ == "__main__":
    main()
