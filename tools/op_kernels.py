#!/usr/bin/env python3
"""Which framework op launched which GPU kernel, with input shapes: one LoRA training step of the
1-layer Llama-3-8B under torch.profiler, kernels grouped by (parent aten / autograd op, shapes).

    python tools/op_kernels.py [--model llama3-8b-1l] [--method lora] [--top 40] [--match SUBSTR]

Prints a markdown table: kernel, the op that launched it (innermost CPU op with shapes), calls,
total / mean device microseconds.  Used to attribute the small hipBLASLt / elementwise kernels of
``tools/prof_bench.sh`` tables to their call sites.
"""
from __future__ import annotations

import argparse
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b-1l")
    ap.add_argument("--method", default="lora")
    ap.add_argument("--batch-size", type=int, default=4)
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--match", default="")
    a = ap.parse_args()

    import torch
    from torch.profiler import ProfilerActivity, profile

    from finetune_controller_amd.train.trainer import TrainConfig, Trainer

    tc = TrainConfig(model=a.model, method=a.method, batch_size=a.batch_size, seq_len=a.seq_len, synthetic=True,
                     max_steps=4, checkpoint_path="/tmp/op_kernels", save_model=False, resume=False, device="cuda",
                     warmup_steps=0)
    tr = Trainer(tc)
    for _ in range(2):
        tr.train_step(1e-4)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        tr.train_step(1e-4)
        torch.cuda.synchronize()
    rows = defaultdict(lambda: [0, 0.0])
    for e in prof.events():
        # CPU ops own the kernels they launched (correlation ids); walk up for context
        if e.device_type.name != "CPU" or not e.kernels:
            continue
        chain, p = [], e
        while p is not None and len(chain) < 3:
            if not p.name.startswith(("hip", "cuda")):
                shapes = [list(s) for s in (p.input_shapes or []) if s]
                chain.append(f"{p.name}{shapes if shapes else ''}")
            p = p.cpu_parent
        site = " <- ".join(chain)
        for k in e.kernels:
            if a.match and a.match not in k.name:
                continue
            r = rows[(k.name[:90], site[:240])]
            r[0] += 1
            r[1] += k.duration
    print(f"# kernels of one {a.model} {a.method} step by launching op (B{a.batch_size} S{a.seq_len})\n")
    print("| us total | calls | us mean | kernel | launched from |")
    print("|---:|---:|---:|---|---|")
    for (k, site), (n, us) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| {us:.0f} | {n} | {us / n:.1f} | `{k}` | {site} |")
    tr.close()


if __name__ == "__main__":
    main()
