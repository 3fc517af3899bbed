#!/usr/bin/env python3
"""Flat AdamW kernel throughput at full-FT scale (csrc/kernels/optim.hip, one-shot grid), bf16 gradients
+ bf16 parameter copy, fp32 master / moments: 28 B per element moved; one JSON line per round (ms, TB/s).
profiles/r4/adamw/ holds the A/B that chose the one-shot 4-wide kernel over the grid-stride loop and an
8-wide group."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    import finetune_controller_amd._C as C

    n = int(float(os.environ.get("N", 2e9)))
    dev = "cuda"
    master = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    param = master.to(torch.bfloat16)
    g = (1e-3 * torch.randn(n, device=dev)).to(torch.bfloat16)
    gs = torch.ones(1, device=dev)
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(3):
        C.adamw_(param, master, m, v, g, 1e-5, 0.9, 0.95, 1e-8, 0.0, 1, gs)
        torch.cuda.synchronize()
        st.record()
        for _ in range(5):
            C.adamw_(param, master, m, v, g, 1e-5, 0.9, 0.95, 1e-8, 0.0, 1, gs)
        en.record()
        torch.cuda.synchronize()
        ms = st.elapsed_time(en) / 5
        print(json.dumps({"kernel": "adamw one-shot", "round": rnd, "n": n, "ms": round(ms, 3),
                          "TBps": round(28 * n / ms / 1e9, 3)}), flush=True)


if __name__ == "__main__":
    main()
