#!/usr/bin/env python3
"""The hand-written projection GEMM (csrc/kernels/gemm_nt.hip) vs hipBLASLt on the base-GEMM shapes of
one Llama-3-8B LoRA step: ``C[T, n] = A[T, k] . B[n, k]^T`` with T = 16384 tokens (4 x 4096), the
augmented LoRA forms of ops/linear.py (k = K + 64 forward, the transposed frozen weight backward).

    python tools/bench_gemm_nt.py [--iters 10] [--rounds 3] [--shapes qkv_fwd,o_fwd]

Ours and the library are timed in INTERLEAVED rounds on the same uniform random [-1, 1) operands (zeros
read fast: DVFS), so box-to-box clock differences cancel; one JSON line per shape with the median
and min ms of each, TF/s on the median, and the max |ours - lib| / max |lib| of one product."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finetune_controller_amd.ops._backend import ext  # noqa: E402
from finetune_controller_amd.ops.gemm import pack_b_nt  # noqa: E402

T = 16384
SHAPES = {  # name: (k, n)
    "qkv_fwd": (4096 + 64, 6144), "o_fwd": (4096 + 64, 4096), "gu_fwd": (4096 + 64, 28672),
    "down_fwd": (14336 + 64, 4096), "down_dx": (4096 + 64, 14336), "gu_dx": (28672 + 64, 4096),
    "o_dx": (4096 + 64, 4096), "qkv_dx": (6144 + 64, 4096), "lm_head": (4096, 4096 * 8),
}


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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    a = ap.parse_args()
    C = ext()
    torch.manual_seed(0)
    for name in a.shapes.split(","):
        k, n = SHAPES[name]
        x = torch.empty(T, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(n, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        y0 = torch.empty(T, n, device="cuda", dtype=torch.bfloat16)
        y1 = torch.empty(T, n, device="cuda", dtype=torch.bfloat16)
        wp = pack_b_nt(w)  # the packed (fragment-order) weight: built once, like a frozen weight's
        assert C.gemm_nt_ok(y1, x, w) and C.gemm_nt_pb_ok(y1, x, wp, n, k), name
        ours, lib, pk = [], [], []
        torch.mm(x, w.t(), out=y0)
        C.gemm_nt_pb_(y1, x, wp, n, k)
        torch.cuda.synchronize()
        err_pk = ((y1.float() - y0.float()).abs().max() / y0.float().abs().max()).item()
        C.gemm_nt_(y1, x, w)
        torch.cuda.synchronize()
        err = ((y1.float() - y0.float()).abs().max() / y0.float().abs().max()).item()
        for _ in range(a.rounds):
            ours.append(timeit(lambda: C.gemm_nt_(y1, x, w), a.iters))
            pk.append(timeit(lambda: C.gemm_nt_pb_(y1, x, wp, n, k), a.iters))
            lib.append(timeit(lambda: torch.mm(x, w.t(), out=y0), a.iters))
        fl = 2.0 * T * n * k
        mo, ml, mp = statistics.median(ours), statistics.median(lib), statistics.median(pk)
        print(json.dumps({"gemm": name, "M": T, "N": n, "K": k,
                          "ours_ms": [round(mo, 3), round(min(ours), 3)], "ours_tf": round(fl / mo / 1e9),
                          "packed_ms": [round(mp, 3), round(min(pk), 3)], "packed_tf": round(fl / mp / 1e9),
                          "lib_ms": [round(ml, 3), round(min(lib), 3)], "lib_tf": round(fl / ml / 1e9),
                          "speedup": round(ml / mo, 3), "speedup_packed": round(ml / mp, 3),
                          "max_rel_err_vs_lib": float(f"{err:.2e}"),
                          "max_rel_err_packed_vs_lib": float(f"{err_pk:.2e}")}), flush=True)
        del x, w, wp, y0, y1
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
