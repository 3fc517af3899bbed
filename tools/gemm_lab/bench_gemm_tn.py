#!/usr/bin/env python3
"""Weight-gradient GEMM dW (+)= dy^T x at the Llama-3-8B full-FT shapes: the hand-written gfx950 TN
kernel (csrc/kernels/gemm_tn.hip) vs hipBLASLt in the layouts the trainer can hand it.

    python tools/bench_gemm_tn.py [--iters 10]

Rows (one JSON line per shape and C dtype): ms and TF/s of
  * ours       -- gemm_tn_(C, dy, x): both operands as stored ([T, out], [T, in]), no copies;
  * lib_tt     -- C.addmm_(dy^T, x): hipBLASLt on the same views;
  * lib_xt     -- C.addmm_(dy^T, (x^T)^T) with x^T materialised beforehand (the trainer's former
                  path); `xt_ms` is the transpose it needs, charged to it in `lib_xt_total_ms`.
Operands are uniform random in [-1, 1) (zeros would read fast: DVFS)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finetune_controller_amd.ops._backend import ext  # noqa: E402

SHAPES = {  # name: (M = out, N = in, K = tokens)
    "qkv": (6144, 4096, 16384),
    "o": (4096, 4096, 16384),
    "gu": (28672, 4096, 16384),
    "down": (4096, 14336, 16384),
    "lm_head_chunk": (128256, 4096, 4096),
}


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--cdtype", default="bf16,fp32")
    a = ap.parse_args()
    from tools.gemm_lab.lab import load

    C = load()
    dev = "cuda"
    for name in a.shapes.split(","):
        M, N, K = SHAPES[name]
        dy = (torch.rand(K, M, device=dev) * 2 - 1).to(torch.bfloat16)
        x = (torch.rand(K, N, device=dev) * 2 - 1).to(torch.bfloat16)
        xt = x.t().contiguous()
        flop = 2.0 * M * N * K
        for cd in a.cdtype.split(","):
            dt = torch.bfloat16 if cd == "bf16" else torch.float32
            c = torch.zeros(M, N, device=dev, dtype=dt)
            ours = timeit(lambda: C.gemm_tn_(c, dy, x, 1.0, 1.0), a.iters)
            if dt == torch.bfloat16:
                tt = timeit(lambda: c.addmm_(dy.t(), x), a.iters)
                xtm = timeit(lambda: c.addmm_(dy.t(), xt.t()), a.iters)
            else:
                tt = timeit(lambda: torch.addmm(c, dy.t(), x, out_dtype=torch.float32, out=c), a.iters)
                xtm = timeit(lambda: torch.addmm(c, dy.t(), xt.t(), out_dtype=torch.float32, out=c), a.iters)
            tr = timeit(lambda: C.transpose2d(x, xt), a.iters)
            # numerics on this shape: one beta=0 product vs the library's
            ref = torch.mm(dy.t(), x).float()
            c0 = torch.empty(M, N, device=dev, dtype=dt)
            C.gemm_tn_(c0, dy, x, 1.0, 0.0)
            err = ((c0.float() - ref).abs().max() / ref.abs().max()).item()
            print(json.dumps({"gemm": name, "c": cd, "M": M, "N": N, "K": K,
                              "ours": [round(ours, 3), round(flop / ours / 1e9)],
                              "lib_tt": [round(tt, 3), round(flop / tt / 1e9)],
                              "lib_xt": [round(xtm, 3), round(flop / xtm / 1e9)],
                              "xt_ms": round(tr, 3), "lib_xt_total_ms": round(xtm + tr, 3),
                              "max_rel_err_vs_lib": float(f"{err:.2e}")}), flush=True)
            del c, c0, ref
        del dy, x, xt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
