#!/usr/bin/env python3
"""Phase cycle counts of the W64 forward from the stamps build (tools/w64_lab/libstamps.so, W64_STAMPS=1):
workgroup 0's first block (the heaviest causal block), tiles 20-23, every wave.  Columns: sync wait, rescale,
X phase (S MFMAs + finish softmax), seam (K reads), Y phase (PV MFMAs + start softmax); ideal X = Y = 32 MFMAs x
32 cycles = 1024."""
import ctypes
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from diag import load  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    L = load(os.path.join(HERE, "libstamps.so"))
    L.ftc_w64_stamps.argtypes = [ctypes.c_void_p]
    B, S, H, KV, D = 4, 4096, 32, 8, 128
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (H + 2 * KV) * D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + KV) * D], qkv[:, (H + KV) * D:]
    o = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for var in (1, 2):
        L.ftc_flash_fwd_config(var)
        for _ in range(3):
            assert L.ftc_flash_fwd(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(), B, S, H, KV,
                                   D, q.stride(0), k.stride(0), o.stride(0), 1 / math.sqrt(D), 1, 0, None, S, st) == 0
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 96)()
        assert L.ftc_w64_stamps(buf) == 0
        bb = (ctypes.c_ulonglong * 192)()
        L.ftc_w64_bstamps.argtypes = [ctypes.c_void_p]
        assert L.ftc_w64_bstamps(bb) == 0
        print(f"variant {var}: block wave | start-loads bodies tail epilogue idle | total (next block start - this)")
        for n in range(8 if var == 1 else 1):
            for w in range(4):
                s = [bb[(n * 4 + w) * 6 + kk] for kk in range(6)]
                d = [s[kk + 1] - s[kk] for kk in range(5)]
                nxt = bb[((n + 1) * 4 + w) * 6] - s[0] if n < 7 and var == 1 else 0
                print(f"  b{n} w{w} | " + " ".join(f"{x:8d}" for x in d) + f" | {s[5] - s[0]} ({nxt})")
        print(f"variant {var}: wave tile | sync rescale X seam Y | total")
        for w in range(4):
            for t in range(4):
                s = [buf[(w * 4 + t) * 6 + kk] for kk in range(6)]
                d = [s[kk + 1] - s[kk] for kk in range(5)]
                print(f"  w{w} t{20 + t} | " + " ".join(f"{x:6d}" for x in d) + f" | {s[5] - s[0]}")


if __name__ == "__main__":
    main()
