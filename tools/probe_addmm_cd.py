#!/usr/bin/env python3
"""Does ``torch.addmm(R, x, W^T, out=D)`` (D != R) run as ONE hipBLASLt call with C = R and D separate,
or as a copy R -> D followed by a beta = 1 GEMM on D?  Times the o-projection shape (T 16384, K 4160,
N 4096) three ways and prints one JSON line; run under ``rocprofv3 --kernel-trace --stats`` to see the
kernels.  (Question behind it: folding the residual add of the decoder layer into the projection GEMM's
epilogue, docs/kernels.md.)"""
import json

import torch


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters, 4)


def main():
    T, K, N = 16384, 4160, 4096
    bf = torch.bfloat16
    x = torch.randn(T, K, device="cuda", dtype=bf)
    w = torch.randn(N, K, device="cuda", dtype=bf)
    r = torch.randn(T, N, device="cuda", dtype=bf)
    d = torch.empty(T, N, device="cuda", dtype=bf)
    fns = {
        "mm": lambda: torch.mm(x, w.t(), out=d),
        "addmm_out": lambda: torch.addmm(r, x, w.t(), out=d),
        "addmm_inplace": lambda: d.addmm_(x, w.t()),
        "copy": lambda: d.copy_(r),
    }
    res = {k: [] for k in fns}
    for _ in range(5):  # interleaved rounds: clock drift hits every arm
        for k, f in fns.items():
            res[k].append(timeit(f))
    out = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    ref = torch.addmm(r.float(), x.float(), w.float().t())
    torch.addmm(r, x, w.t(), out=d)
    out["max_rel_err"] = float((d.float() - ref).abs().max() / ref.abs().max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
