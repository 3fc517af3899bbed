#!/usr/bin/env python3
"""The LoRA "tail" product ``x[:, K:K+Rp] = x[:, :K] . Bm^T`` at the Llama-3-8B step's shapes (T = 16384,
row stride K + 64): the HIP streaming kernel (csrc/kernels/swiglu_lora.hip ``tail_gemm``) vs hipBLASLt
writing the same strided tail (ops/linear.py ``tail_product``'s fallback).  Interleaved rounds; one JSON
line per shape with median ms, the kernel's HBM rate over x, and the max |ours - lib| / max |lib|.

    python tools/bench_tail_gemm.py [--rounds 5] [--iters 20]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finetune_controller_amd.ops._backend import ext  # noqa: E402

T = 16384
# (name, K, nct): o-proj / down-proj tails (r 16), the gate|up A pair (32), the packed q|k|v forward (48) and
# its input-gradient tail over the 6144-wide q|k|v output gradient
SHAPES = (("o_fwd", 4096, 1), ("gu_fwd", 4096, 2), ("qkv_fwd", 4096, 3), ("qkv_dx", 6144, 3))


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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C = ext()
    torch.manual_seed(0)
    Rp = 64
    for name, K, nct in SHAPES:
        x = torch.empty(T, K + Rp, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        bm = torch.zeros(Rp, K, device="cuda", dtype=torch.bfloat16)
        bm[: 16 * nct] = 0.05 * torch.randn(16 * nct, K, device="cuda", dtype=torch.bfloat16)
        xv, tail = x[:, :K], x[:, K:]

        def ours():
            C.tail_gemm_(xv, bm, nct, Rp)

        def lib():
            torch.mm(xv, bm.t(), out=tail)

        ours()
        ref_ours = tail.clone()
        lib()
        ref_lib = tail.clone()
        torch.cuda.synchronize()
        t_o, t_l = [], []
        for _ in range(a.rounds):
            t_o.append(timeit(ours, a.iters))
            t_l.append(timeit(lib, a.iters))
        mo, ml = statistics.median(t_o), statistics.median(t_l)
        err = float((ref_ours.float() - ref_lib.float()).abs().max() / ref_lib.float().abs().max().clamp_min(1e-30))
        print(json.dumps({"shape": name, "K": K, "nct": nct, "ours_ms": round(mo, 4), "lib_ms": round(ml, 4),
                          "ours_TBps": round(T * K * 2 / mo / 1e9, 2), "speedup": round(ml / mo, 3),
                          "max_rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
