#!/usr/bin/env python3
"""lm_head GEMM orientations at the Llama-3-8B CE chunk shape (hipBLASLt through torch.mm).

    python tools/bench_lm_head.py [--rows 4096]

forward   logits [T, V] = h [T, K] . W^T        (current)    vs   logits^T [V, T] = W . h^T
backward  dh [T, K] = dlogits [T, V] . W (NN / W^T copy)     vs   dh = (dlogits^T)^T . W  (from logits^T)
Interleaved rounds; prints one JSON line per orientation with ms and TFLOP/s.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, iters=10):
    fn()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    T, K, V = a.rows, 4096, 128256
    bf = torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    h = torch.randn(T, K, device="cuda", dtype=bf, generator=g)
    hT = h.t().contiguous()
    W = torch.randn(V, K, device="cuda", dtype=bf, generator=g) * 0.02
    WT = W.t().contiguous()
    logits = torch.empty(T, V, device="cuda", dtype=bf)
    logitsT = torch.empty(V, T, device="cuda", dtype=bf)
    dh = torch.empty(T, K, device="cuda", dtype=bf)
    fl = 2 * T * K * V
    cases = {
        "fwd h.W^T -> [T,V]": lambda: torch.mm(h, W.t(), out=logits),
        "fwd W.h^T -> [V,T] (h^T view)": lambda: torch.mm(W, h.t(), out=logitsT),
        "fwd W.h^T -> [V,T] (h^T copy)": lambda: torch.mm(W, hT, out=logitsT),
        "bwd dl.W (NN)": lambda: torch.mm(logits, W, out=dh),
        "bwd dl.W (W^T copy)": lambda: torch.mm(logits, WT.t(), out=dh),
        "bwd (dl^T)^T.W": lambda: torch.mm(logitsT.t(), W, out=dh),
        "bwd (dl^T)^T.W (W^T copy)": lambda: torch.mm(logitsT.t(), WT.t(), out=dh),
    }
    res = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, fn in cases.items():
            res[k].append(timeit(fn))
    for k, v in res.items():
        ms = min(v)
        print(json.dumps({"case": k, "rows": T, "ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
