#!/usr/bin/env python3
"""Flash-attention forward variants (csrc/kernels/flash_attn_fwd.hip: QB1 = 32 query rows per wave, two
workgroups per CU; QB2 = two 32-row blocks per wave, one workgroup per CU) at the Llama-3-8B layer shape,
interleaved rounds in one process on random data; one JSON line per variant with ms, TF/s (causal FLOPs)
and the max |difference| to QB1's output and LSE.

    python tools/bench_attn_fwd.py [--B 4 --S 4096 --H 32 --KV 8 --D 128] [--rounds 5 --iters 20]"""
import argparse
import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finetune_controller_amd.ops._backend import ext  # noqa: E402


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
    for k, v in (("B", 4), ("S", 4096), ("H", 32), ("KV", 8), ("D", 128), ("rounds", 5), ("iters", 20), ("window", 0)):
        ap.add_argument(f"--{k}", type=int, default=v)
    a = ap.parse_args()
    C = ext()
    B, S, H, KV, D = a.B, a.S, a.H, a.KV, a.D
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (H + 2 * KV) * D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + KV) * D], qkv[:, (H + KV) * D:]
    scale = 1 / math.sqrt(D)
    outs, times = {}, {1: [], 2: []}
    for qb in (1, 2):
        C.flash_fwd_config(qb)
        outs[qb] = [t.clone() for t in C.flash_fwd(q, k, v, B, S, H, KV, D, scale, True, a.window)]
    for _ in range(a.rounds):
        for qb in (1, 2):
            C.flash_fwd_config(qb)
            times[qb].append(timeit(lambda: C.flash_fwd(q, k, v, B, S, H, KV, D, scale, True, a.window), a.iters))
    C.flash_fwd_config(1)
    fl = 4 * B * H * S * S * D / 2
    for qb in (1, 2):
        ms = statistics.median(times[qb])
        do = (outs[qb][0].float() - outs[1][0].float()).abs().max().item()
        dl = (outs[qb][1] - outs[1][1]).abs().max().item()
        print(json.dumps({"variant": f"qb{qb}", "ms": round(ms, 4), "min_ms": round(min(times[qb]), 4),
                          "tf": round(fl / ms / 1e9), "max_abs_diff_o": do, "max_abs_diff_lse": dl}), flush=True)


if __name__ == "__main__":
    main()
