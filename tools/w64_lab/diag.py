#!/usr/bin/env python3
"""Numerics of the lab builds of the flash forward (tools/w64_lab/build.sh) vs an fp32 reference."""
import ctypes
import glob
import math
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def load(path):
    L = ctypes.CDLL(path)
    L.ftc_flash_fwd.restype = ctypes.c_int
    L.ftc_flash_fwd.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int] * 5 + [ctypes.c_longlong] * 3 + \
        [ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    L.ftc_flash_fwd_config.argtypes = [ctypes.c_int]
    return L


def ref(q, k, v, B, S, H, KV, D, causal):
    G = H // KV
    qf = q.float().view(B, S, H, D).transpose(1, 2)
    kf = k.float().view(B, S, KV, D).transpose(1, 2).repeat_interleave(G, 1)
    vf = v.float().view(B, S, KV, D).transpose(1, 2).repeat_interleave(G, 1)
    s = qf @ kf.transpose(-1, -2) / math.sqrt(D)
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=q.device), 1), float("-inf"))
    return (torch.softmax(s, -1) @ vf).transpose(1, 2).reshape(B * S, H * D)


def main():
    libs = {os.path.basename(p)[3:-3]: load(p) for p in sorted(glob.glob(os.path.join(HERE, "lib*.so")))}
    D = 128
    for (B, S, H, KV, causal) in [(2, 256, 8, 2, True), (1, 256, 4, 4, False), (1, 512, 2, 1, True)]:
        torch.manual_seed(0)
        qkv = torch.randn(B * S, (H + 2 * KV) * D, device="cuda", dtype=torch.bfloat16)
        q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + KV) * D], qkv[:, (H + KV) * D:]
        r = ref(q, k, v, B, S, H, KV, D, causal)
        line = [f"B{B} S{S} H{H} KV{KV} c={int(causal)}"]
        for name, L in libs.items():
            for var in (1, 0) if name == "base" else (1,):
                L.ftc_flash_fwd_config(var)
                o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
                lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
                rc = L.ftc_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, H, KV,
                                     D, q.stride(0), k.stride(0), o.stride(0), 1 / math.sqrt(D), int(causal), 0, None, S,
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                torch.cuda.synchronize()
                d = (o.float() - r).abs().view(B * S, H, D).amax(-1)
                line.append(f"{name}{'' if var else '/w32'}: rc={rc} max {d.max().item():.3f} bad {(d > 0.05).sum().item()}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
