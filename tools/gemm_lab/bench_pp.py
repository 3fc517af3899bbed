#!/usr/bin/env python3
"""Lab bench for the 8-wave ping-pong projection GEMM (tools/gemm_lab/gemm_pp.hip, built by
tools/gemm_lab/build.sh into tools/gemm_lab/libgemm_pp.so): correctness against an fp32 / exact-integer
reference on small and production shapes, then interleaved timing rounds (same uniform random [-1, 1)
operands) of hipBLASLt (torch.mm), the lab 4-wave kernel (tools/gemm_lab/lab.py gemm_nt_) and the ping-pong kernel on
the Llama-3-8B LoRA-step shapes (T = 16384).  One JSON line per shape.

    python tools/gemm_lab/bench_pp.py [--variants d0,d3,m1] [--shapes qkv_fwd,o_fwd] [--iters 20] [--rounds 5]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from finetune_controller_amd.ops._backend import ext  # noqa: E402

T = 16384
SHAPES = {  # name: (k, n) -- as tools/bench_gemm_nt.py
    "qkv_fwd": (4096 + 64, 6144), "o_fwd": (4096 + 64, 4096), "gu_fwd": (4096 + 64, 28672),
    "down_fwd": (14336 + 64, 4096), "down_dx": (4096 + 64, 14336), "gu_dx": (28672 + 64, 4096),
    "o_dx": (4096 + 64, 4096), "qkv_dx": (6144 + 64, 4096), "lm_head": (4096, 4096 * 8),
}

def _load(mode):
    lib = ctypes.CDLL(os.path.join(HERE, f"libgemm_pp_{mode}.so"))
    lib.ftc_gemm_pp.restype = ctypes.c_int
    lib.ftc_gemm_pp.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong,
                                ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    return lib


_libs = {}


def pp(c, a, b, alpha=1.0, grid_cap=0, group=-8, xcc=32, mode="d0"):
    M, K = a.shape
    N = b.shape[0]
    rc = _libs[mode].ftc_gemm_pp(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(), c.stride(0), M, N, K,
                          alpha, grid_cap, group, xcc, torch.cuda.current_stream().cuda_stream)
    if rc != 0:
        raise RuntimeError(f"ftc_gemm_pp rc={rc} for {M}x{N}x{K}")


def check(mode):
    torch.manual_seed(3)
    cases = [(256, 256, 64, 0, 0), (512, 768, 192, 0, 0), (1024, 1280, 448, 8, 3), (768, 512, 128, 0, 1),
             (2048, 2048, 4160, 0, 0), (1024, 768, 64, 0, 5)]
    for M, N, K, pad, cap in cases:
        abuf = torch.randint(-3, 4, (M, K + pad), device="cuda").to(torch.bfloat16)
        a = abuf[:, :K]
        b = (torch.arange(N * K, device="cuda").reshape(N, K) % 7 - 3).to(torch.bfloat16)
        c = torch.full((M, N), 7.0, device="cuda", dtype=torch.bfloat16)
        pp(c, a, b, grid_cap=cap, mode=mode)
        exact = (a.double() @ b.double().t()).to(torch.bfloat16)
        ok = torch.equal(c, exact)
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        pp(c, a, b, alpha=0.5, grid_cap=cap, mode=mode)
        ref = 0.5 * (a.float() @ b.float().t())
        err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps({"check": [M, N, K, pad, cap], "variant": mode, "exact_int": ok, "max_rel_err": float(f"{err:.2e}")}), flush=True)
        if not ok or err > 2e-2:
            raise SystemExit("ping-pong GEMM mismatch")


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
    ap.add_argument("--shapes", default="qkv_fwd,o_fwd,gu_fwd,down_dx,down_fwd")
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the correctness cases (counter runs)")
    ap.add_argument("--variants", default="d0",
                    help="ping-pong builds to time (tools/gemm_lab/build.sh): d0-d3 DMA placements, m1-m3 ablations of d0")
    a = ap.parse_args()
    modes = a.variants.split(",")
    for m in modes:
        _libs.setdefault(m, _load(m))
    for m in modes:
        if m.startswith("d") and not a.no_check:
            check(m)
    if a.check_only:
        return
    from tools.gemm_lab.lab import load

    C = load()
    torch.manual_seed(0)
    for name in a.shapes.split(","):
        k, n = SHAPES[name]
        x = torch.empty(T, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(n, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        y0 = torch.empty(T, n, device="cuda", dtype=torch.bfloat16)
        y1 = torch.empty_like(y0)
        y2 = torch.empty_like(y0)
        y3 = torch.empty_like(y0)
        torch.mm(x, w.t(), out=y0)
        C.gemm_nt_(y1, x, w)
        errs = {}
        for m in modes:
            if m.startswith("d"):
                y2.zero_()
                pp(y2, x, w, mode=m)
                torch.cuda.synchronize()
                errs[m] = float(f"{((y2.float() - y0.float()).abs().max() / y0.float().abs().max()).item():.2e}")
        arms = {"lib": lambda: torch.mm(x, w.t(), out=y0), "nt4": lambda: C.gemm_nt_(y1, x, w)}
        for m in modes:
            arms[m] = (lambda m_: (lambda: pp(y2 if m_.startswith("d") else y3, x, w, mode=m_)))(m)
        t = {k_: [] for k_ in arms}
        for _ in range(a.rounds):
            for k_, f in arms.items():
                t[k_].append(timeit(f, a.iters))
        fl = 2.0 * T * n * k
        med = {k_: statistics.median(v) for k_, v in t.items()}
        print(json.dumps({"gemm": name, "M": T, "N": n, "K": k,
                          **{f"{k_}_ms": round(v, 4) for k_, v in med.items()},
                          **{f"{k_}_tf": round(fl / v / 1e9) for k_, v in med.items()},
                          **{f"{k_}_vs_lib": round(med["lib"] / v, 4) for k_, v in med.items() if k_ != "lib"},
                          "max_rel_err_vs_lib": errs}), flush=True)
        del x, w, y0, y1, y2, y3
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
