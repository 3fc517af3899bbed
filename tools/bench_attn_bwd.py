#!/usr/bin/env python3
"""Flash-attention backward dK/dV variants (csrc/kernels/flash_attn_bwd.hip: "8" = 8 waves x 32 keys with the
ping-pong phase order, the default; "il" = 4 waves x 64 keys with the fenced in-wave interleave) at the
Llama-3-8B layer shape, interleaved rounds in one process on random data.  Times the whole backward call
(delta + dK/dV + dQ); one JSON line per variant with ms and the max |difference| of dQ / dK / dV to the
default's.

    python tools/bench_attn_bwd.py [--B 4 --S 4096 --H 32 --KV 8 --D 128] [--rounds 5 --iters 10]"""
import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finetune_controller_amd.ops._backend import ext  # noqa: E402

VARIANTS = {"8": 8, "4": 4, "il": 1}


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
    for k, v in (("B", 4), ("S", 4096), ("H", 32), ("KV", 8), ("D", 128), ("rounds", 5), ("iters", 10), ("window", 0)):
        ap.add_argument(f"--{k}", type=int, default=v)
    a = ap.parse_args()
    C = ext()
    B, S, H, KV, D = a.B, a.S, a.H, a.KV, a.D
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (H + 2 * KV) * D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + KV) * D], qkv[:, (H + KV) * D:]
    scale = 1 / math.sqrt(D)
    o, lse = C.flash_fwd(q, k, v, B, S, H, KV, D, scale, True, a.window)
    do = torch.randn_like(o)
    dq = torch.empty_like(q.contiguous())
    dk = torch.empty(B * S, KV * D, device="cuda", dtype=torch.bfloat16)
    dv = torch.empty_like(dk)

    def run():
        C.flash_bwd(q, k, v, o, do, lse, dq, dk, dv, B, S, H, KV, D, scale, True, a.window, None, None, 0,
                    None, None, None)

    outs, times = {}, {n: [] for n in VARIANTS}
    for n, w in VARIANTS.items():
        C.flash_dkdv_config(w)
        run()
        torch.cuda.synchronize()
        outs[n] = (dq.clone(), dk.clone(), dv.clone())
    for _ in range(a.rounds):
        for n, w in VARIANTS.items():
            C.flash_dkdv_config(w)
            times[n].append(timeit(run, a.iters))
    C.flash_dkdv_config(8)
    for n in VARIANTS:
        ms = statistics.median(times[n])
        diff = [(x.float() - y.float()).abs().max().item() for x, y in zip(outs[n], outs["8"])]
        print(json.dumps({"variant": n, "bwd_ms": round(ms, 4), "min_ms": round(min(times[n]), 4),
                          "max_abs_diff_dq_dk_dv": diff}), flush=True)


if __name__ == "__main__":
    main()
