#!/usr/bin/env python3
"""Full-FT weight gradients dW (+)= dy^T x at the Llama-3-8B shapes (T = 16384 tokens): the production
path (x transposed by transpose.hip, then one hipBLASLt GEMM) against split-K decompositions that turn
the wave-quantised tile grids (qkv 384 tiles of 256 x 256 = 1.5 waves on 256 CUs, down 896 = 3.5)
into whole waves: ONE batched GEMM over the K halves / quarters into fp32 partials, then one pass that
sums them into C.  Interleaved rounds, one line per shape:

    python tools/bench_dw_split.py [--shapes qkv,o,gu,down] [--rounds 5] [--iters 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def lab():
    from tools.gemm_lab.lab import load

    return load()

from finetune_controller_amd.ops import linear as L  # noqa: E402

T = 16384
SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gu": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="qkv,o,gu,down")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.manual_seed(0)
    for name in a.shapes.split(","):
        M, N = SHAPES[name]
        dy = torch.empty(T, M, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        x = torch.empty(T, N, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        xt = torch.empty(N, T, device="cuda", dtype=torch.bfloat16)
        c = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
        ref = torch.mm(dy.t().float(), x.float()) if M * N <= 6144 * 4096 else None
        parts = {s: torch.empty(s, M, N, device="cuda", dtype=torch.float32) for s in (2, 4)}
        parts_bf = torch.empty(2, M, N, device="cuda", dtype=torch.bfloat16)

        def base():
            L.transpose2d(x, xt)
            torch.mm(dy.t(), xt.t(), out=c)

        def split(s, fp32=True):
            def run():
                L.transpose2d(x, xt)
                k = T // s
                A = dy.as_strided((s, M, k), (k * M, 1, M))
                B = xt.as_strided((s, k, N), (k, 1, T))
                if fp32:
                    p = parts[s]
                    torch.bmm(A, B, out_dtype=torch.float32, out=p)
                else:
                    p = parts_bf
                    torch.bmm(A, B, out=p)
                torch.sum(p, 0, out=c) if not fp32 else c.copy_(p.sum(0))
            return run

        def split_tt(s):  # no transposed copy: x as stored ("TT" form) into the batched GEMM
            def run():
                k = T // s
                A = dy.as_strided((s, M, k), (k * M, 1, M))
                B = x.as_strided((s, k, N), (k * N, N, 1))
                p = parts[s]
                torch.bmm(A, B, out_dtype=torch.float32, out=p)
                c.copy_(p.sum(0))
            return run

        from finetune_controller_amd.ops._backend import ext

        def split_hip(s):  # the production path (ops.linear.wgrad_mm): batched GEMM + HIP partial sum
            def run():
                L.transpose2d(x, xt)
                k = T // s
                A = dy.as_strided((s, M, k), (k * M, 1, M))
                B = xt.as_strided((s, k, N), (k, 1, T))
                p = parts[s]
                torch.bmm(A, B, out_dtype=torch.float32, out=p)
                ext().splitk_sum_(c, p, 0.0)
            return run

        def tn(s):  # the hand-written TN kernel (operands as stored, no transposed copy), split s ways
            def run():
                if s == 1:
                    lab().gemm_tn_(c, dy, x, 1.0, 0.0)
                else:
                    p = parts[s]
                    lab().gemm_tn_split_(p, dy, x)
                    ext().splitk_sum_(c, p, 0.0)
            return run

        arms = {"base": base, "tn1": tn(1), "tn2": tn(2), "tn4": tn(4), "split2_hip": split_hip(2), "wgrad_mm": lambda: L.wgrad_mm(c, dy.t(), L.transpose2d(x, xt).t(), 0.0), "split2": split(2), "split4": split(4), "split2_bf16": split(2, False),
                "split2_tt": split_tt(2)}
        errs = {}
        for k, fn in arms.items():
            fn()
            torch.cuda.synchronize()
            if ref is not None:
                errs[k] = round(((c.float() - ref).norm() / ref.norm()).item(), 6)
        times = {k: [] for k in arms}
        for _ in range(a.rounds):
            for k, fn in arms.items():
                times[k].append(timeit(fn, a.iters))
        flops = 2.0 * M * N * T
        out = {"gemm": name, "M": M, "N": N, "K": T}
        for k, v in times.items():
            ms = min(v)
            out[k] = [round(ms, 4), round(flops / ms / 1e9)]
        out["rel_err_vs_fp32"] = errs
        print(json.dumps(out), flush=True)
        del dy, x, xt, c, parts, parts_bf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
