#!/usr/bin/env python3
"""Attention microbenchmark at the flagship shape: our gfx950 flash kernels vs torch SDPA (AOTriton).

Llama-3-8B attention per layer at micro-batch 4 x 4096: H=32, KV=8, D=128, causal.  Interleaved
rounds in one process (guide §5.4 rule 24), random gaussian data (rule 25).  Prints JSON lines.
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timeit(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=4096)
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--KV", type=int, default=8)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--window", type=int, default=0)
    ap.add_argument("--doc-len", type=int, default=0, help="packed documents of this many tokens (0: one per row)")
    a = ap.parse_args()
    from finetune_controller_amd.ops.attention import _FlashPacked, _sdpa_packed, segments_from_eos

    B, S, H, KV, D = a.B, a.S, a.H, a.KV, a.D
    dev = "cuda"
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (H + 2 * KV) * D, device=dev, dtype=torch.bfloat16)
    do = torch.randn(B * S, H * D, device=dev, dtype=torch.bfloat16)
    scale = 1 / math.sqrt(D)
    flops_fwd = 4 * B * H * S * S * D / 2  # causal
    seg = None
    if a.doc_len:
        ids = torch.zeros(B, S, dtype=torch.long, device=dev)
        ids[:, a.doc_len - 1::a.doc_len] = 2
        seg = segments_from_eos(ids, 2)
    x1 = qkv.clone().requires_grad_(True)
    x2 = qkv.clone().requires_grad_(True)

    def ours_fwd():
        return _FlashPacked.apply(x1, B, S, H, KV, D, True, a.window, scale, 0, 0, seg)

    def sdpa_fwd():
        return _sdpa_packed(x2, B, S, H, KV, D, True, a.window, scale, seg)

    def ours_fb():
        ours_fwd().backward(do)

    def sdpa_fb():
        sdpa_fwd().backward(do)

    for f in (ours_fwd, sdpa_fwd, ours_fb, sdpa_fb):
        f()
    torch.cuda.synchronize()
    res = {"ours_fwd": [], "sdpa_fwd": [], "ours_fwdbwd": [], "sdpa_fwdbwd": []}
    with torch.no_grad():
        pass
    for _ in range(a.rounds):
        with torch.no_grad():
            res["ours_fwd"].append(timeit(lambda: _FlashPacked.apply(qkv, B, S, H, KV, D, True, a.window, scale, 0, 0,
                                                                     seg), a.iters))
            res["sdpa_fwd"].append(timeit(lambda: _sdpa_packed(qkv, B, S, H, KV, D, True, a.window, scale, seg),
                                          a.iters))
        res["ours_fwdbwd"].append(timeit(ours_fb, a.iters))
        res["sdpa_fwdbwd"].append(timeit(sdpa_fb, a.iters))
    out = {"shape": dict(B=B, S=S, H=H, KV=KV, D=D, causal=True, window=a.window, doc_len=a.doc_len)}
    for k, v in res.items():
        ms = min(v)
        fl = flops_fwd * (1 if "bwd" not in k else 3.5)
        out[k] = {"ms": round(ms, 3), "tflops": round(fl / ms / 1e9, 1)}
    out["bwd_only_ms"] = {"ours": round(out["ours_fwdbwd"]["ms"] - out["ours_fwd"]["ms"], 3),
                          "sdpa": round(out["sdpa_fwdbwd"]["ms"] - out["sdpa_fwd"]["ms"], 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
