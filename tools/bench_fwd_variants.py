#!/usr/bin/env python3
"""Flash forward variants A/B at the Llama-3-8B layer shape (B4 S4096 H32 KV8 D128 causal), interleaved
rounds in one process on gaussian data (guide §5.4 rules 24/25): 1 = W64 (one wave per SIMD, 64 rows per
wave), 0 = the 32-row kernel.  Prints one JSON line per variant with ms / TF/s and the max |diff| of O and
LSE against variant 0."""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--S", type=int, default=4096)
    ap.add_argument("--H", type=int, default=32)
    ap.add_argument("--KV", type=int, default=8)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--noncausal", action="store_true")
    a = ap.parse_args()
    import finetune_controller_amd._C as C

    B, S, H, KV, D = a.B, a.S, a.H, a.KV, 128
    causal = not a.noncausal
    torch.manual_seed(0)
    qkv = torch.randn(B * S, (H + 2 * KV) * D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + KV) * D], qkv[:, (H + KV) * D:]
    scale = 1 / math.sqrt(D)
    flops = 4 * B * H * S * S * D / (2 if causal else 1)
    outs, times = {}, {0: [], 1: [], 2: []}
    for var in (0, 1, 2):
        C.flash_fwd_config(var)
        outs[var] = C.flash_fwd(q, k, v, B, S, H, KV, D, scale, causal, 0)
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for var in (1, 2, 0):
            C.flash_fwd_config(var)
            st.record()
            for _ in range(a.iters):
                C.flash_fwd(q, k, v, B, S, H, KV, D, scale, causal, 0)
            en.record()
            torch.cuda.synchronize()
            times[var].append(st.elapsed_time(en) / a.iters)
    C.flash_fwd_config(-1)
    for var in (1, 2, 0):
        ms = sorted(times[var])[len(times[var]) // 2]
        do = (outs[var][0].float() - outs[0][0].float()).abs().max().item()
        dl = (outs[var][1] - outs[0][1]).abs().max().item()
        print(json.dumps({"variant": {0: "w32", 1: "w64-persistent", 2: "w64-per-block"}[var], "ms_median": round(ms, 4), "ms_min": round(min(times[var]), 4),
                          "tflops": round(flops / ms / 1e9, 1), "max_abs_diff_o_vs_w32": do, "max_abs_diff_lse_vs_w32": dl,
                          "shape": dict(B=B, S=S, H=H, KV=KV, D=D, causal=causal)}), flush=True)


if __name__ == "__main__":
    main()
