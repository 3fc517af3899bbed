#!/usr/bin/env python3
"""The hand-written projection GEMM (csrc/kernels/gemm_nt.hip) vs hipBLASLt on the base-GEMM shapes of
one Llama-3-8B LoRA step: ``C[T, n] = A[T, k] . B[n, k]^T`` with T = 16384 tokens (4 x 4096), the
augmented LoRA forms of ops/linear.py (k = K + 64 forward, the transposed frozen weight backward).

    python tools/bench_gemm_nt.py [--iters 20] [--rounds 5] [--shapes qkv_fwd,o_fwd] \
        [--configs "0,-8,32;0,16,2"]

Each config is ``grid_cap,group,xcc`` (GemmLab.gemm_nt_config: grid_cap 0 = one persistent workgroup per CU,
a large cap = one workgroup per tile; group > 0 M-fast / < 0 N-fast tile groups; xcc logical ids per XCD
slot).  Every config and the library are timed in
INTERLEAVED rounds on the same uniform random [-1, 1) operands (zeros read fast: DVFS), so box-to-box
clock differences cancel; one JSON line per (shape, config) with the median / min ms, TF/s on the
median, the speed-up over the library and the max |ours - lib| / max |lib| of one product."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from finetune_controller_amd.ops._backend import ext  # noqa: E402

T = 16384
SHAPES = {  # name: (k, n)
    "qkv_fwd": (4096 + 64, 6144), "o_fwd": (4096 + 64, 4096), "gu_fwd": (4096 + 64, 28672),
    "down_fwd": (14336 + 64, 4096), "down_dx": (4096 + 64, 14336), "gu_dx": (28672 + 64, 4096),
    "o_dx": (4096 + 64, 4096), "qkv_dx": (6144 + 64, 4096), "lm_head": (4096, 4096 * 8),
}
DEFAULT_CONFIGS = "0,-8,32"


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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--configs", default=DEFAULT_CONFIGS)
    ap.add_argument("--T", type=int, default=T)
    a = ap.parse_args()
    from tools.gemm_lab.lab import load

    C = load()
    cfgs = [tuple(int(v) for v in c.split(",")) for c in a.configs.split(";") if c.strip()]
    torch.manual_seed(0)
    for name in a.shapes.split(","):
        k, n = SHAPES[name]
        x = torch.empty(a.T, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(n, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        y0 = torch.empty(a.T, n, device="cuda", dtype=torch.bfloat16)
        y1 = torch.empty(a.T, n, device="cuda", dtype=torch.bfloat16)
        assert C.gemm_nt_ok(y1, x, w), name
        torch.mm(x, w.t(), out=y0)
        errs = []
        for cfg in cfgs:
            C.gemm_nt_config(*cfg)
            y1.zero_()
            C.gemm_nt_(y1, x, w)
            torch.cuda.synchronize()
            errs.append(((y1.float() - y0.float()).abs().max() / y0.float().abs().max()).item())
        ours = [[] for _ in cfgs]
        lib = []
        for _ in range(a.rounds):
            for i, cfg in enumerate(cfgs):
                C.gemm_nt_config(*cfg)
                ours[i].append(timeit(lambda: C.gemm_nt_(y1, x, w), a.iters))
            lib.append(timeit(lambda: torch.mm(x, w.t(), out=y0), a.iters))
        fl = 2.0 * a.T * n * k
        ml = statistics.median(lib)
        for i, cfg in enumerate(cfgs):
            mo = statistics.median(ours[i])
            print(json.dumps({"gemm": name, "M": a.T, "N": n, "K": k, "config": list(cfg),
                              "ours_ms": [round(mo, 4), round(min(ours[i]), 4)], "ours_tf": round(fl / mo / 1e9),
                              "lib_ms": [round(ml, 4), round(min(lib), 4)], "lib_tf": round(fl / ml / 1e9),
                              "speedup": round(ml / mo, 4), "max_rel_err_vs_lib": float(f"{errs[i]:.2e}")}),
                  flush=True)
        del x, w, y0, y1
        torch.cuda.empty_cache()
    C.gemm_nt_config(*[int(v) for v in DEFAULT_CONFIGS.split(",")])


if __name__ == "__main__":
    main()
