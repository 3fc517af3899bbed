#!/usr/bin/env python3
"""All-reduce bus-bandwidth sweep over xGMI: torch ProcessGroupNCCL (RCCL) vs the
native engine (csrc/comm), bf16, message sizes 1 MB .. 1 GB.  Picks the DDP bucket size.

Run one rank per GPU:
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29510 \
      tools/comm_bench.py [--max-mb 1024]
Rank 0 prints one JSON line per (engine, size): algbw = bytes / t, busbw = algbw * 2 (n-1) / n.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from finetune_controller_amd.parallel.dist import init_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-mb", type=float, default=1)
    ap.add_argument("--max-mb", type=float, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    info = init_distributed()
    n = info.world_size
    native = None
    if info.device.type == "cuda" and n > 1:
        from finetune_controller_amd.parallel.comm import NativeComm

        native = NativeComm()
    mb = a.min_mb
    while mb <= a.max_mb:
        numel = int(mb * 2**20 / 2)
        t = torch.ones(numel, device=info.device, dtype=torch.bfloat16)
        res = {}
        for name in ("torch", "native"):
            if name == "native" and native is None:
                continue
            if name == "native":
                sec = native.bench_all_reduce(t, a.iters)
            else:
                dist.all_reduce(t)
                if info.device.type == "cuda":
                    torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    dist.all_reduce(t)
                if info.device.type == "cuda":
                    torch.cuda.synchronize()
                sec = (time.perf_counter() - t0) / a.iters
            algbw = numel * 2 / sec / 1e9
            res[name] = {"ms": round(sec * 1e3, 3), "algbw_GBps": round(algbw, 1),
                         "busbw_GBps": round(algbw * 2 * (n - 1) / max(n, 1), 1)}
        if info.rank == 0:
            print(json.dumps({"n_gpus": n, "size_mb": mb, **res}), flush=True)
        mb *= 2
    if native is not None:
        native.close()
    if n > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
