#!/usr/bin/env python3
"""Headline benchmark: fine-tune tokens/sec for the whole node, Llama-3-8B LoRA (BASELINE.json).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU (RCCL over xGMI for N > 1).  Each rank trains the FULL Llama-3-8B architecture
(random-init bf16 weights, synthetic uniform token ids) with LoRA r=16 / alpha=32 on all seven
linear projections of every layer -- forward, backward, bucketed gradient all-reduce overlapped
with backward, global grad-norm clip and the AdamW update are all inside the timed region.
Weak scaling: the per-GPU micro-batch is fixed, so global batch = micro_batch x N.

W untimed warmup steps, then K steps bracketed by barrier + device synchronize on both sides; the
elapsed time is the MAX over ranks; rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_METRIC = "fine-tune tokens/sec (whole node), Llama-3-8B LoRA at 1/2/4/8 MI355X"


def _mark(op: str):
    import torch

    try:
        if op == "push":
            torch.cuda.nvtx.range_push("ftc_timed")
        else:
            torch.cuda.nvtx.range_pop()
    except Exception:  # no roctx in this build: profiles fall back to whole-run stats
        pass


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--method", default="lora", choices=["lora", "qlora", "full"])
    ap.add_argument("--batch-size", type=int, default=int(os.environ.get("FTC_BENCH_MICRO", "4")))
    ap.add_argument("--seq-len", type=int, default=int(os.environ.get("FTC_BENCH_SEQ", "4096")))
    ap.add_argument("--lora-r", type=int, default=16)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--comm-engine", default="torch", choices=["torch", "native"])
    ap.add_argument("--zero-stage", type=int, default=0, choices=[0, 1],
                    help="1: ZeRO-1 -- AdamW state sharded over the data-parallel ranks (reduce-scatter + all-gather)")
    ap.add_argument("--checkpoint-layers", action="store_true")
    ap.add_argument("--ce-chunk-rows", type=int, default=int(os.environ.get("FTC_CE_CHUNK", "4096")),
                    help="rows per lm_head + cross-entropy chunk (the only vocab-sized buffer)")
    ap.add_argument("--kernels", default=None, choices=["hip", "torch"],
                    help="torch = stock PyTorch-ROCm ops (the 'before' row)")
    ap.add_argument("--graph", action="store_true", help="whole training step captured in a hipGraph (1 GPU)")
    ap.add_argument("--doc-len", type=int, default=0,
                    help="packed documents of this many tokens (document-masked attention; 0: one per row)")
    ap.add_argument("--profile-steps", type=int, default=0, help="extra steps under torch.profiler (not timed)")
    a = ap.parse_args(argv)
    if a.kernels:
        os.environ["FTC_KERNELS"] = a.kernels

    import torch

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from finetune_controller_amd.parallel import dist as pdist
    from finetune_controller_amd.train.trainer import TrainConfig, Trainer

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != a.gpus:
        print(f"[bench] warning: --gpus {a.gpus} but WORLD_SIZE={world_env}; using WORLD_SIZE", file=sys.stderr)

    tc = TrainConfig(model=a.model, method=a.method, lora_r=a.lora_r, lora_alpha=2.0 * a.lora_r,
                     batch_size=a.batch_size, seq_len=a.seq_len, synthetic=True, max_steps=a.warmup + a.steps,
                     warmup_steps=0, schedule="constant", lr=1e-4, bucket_mb=a.bucket_mb, comm_engine=a.comm_engine, zero_stage=a.zero_stage,
                     checkpoint_layers=a.checkpoint_layers, ce_chunk_rows=a.ce_chunk_rows, save_model=False, resume=False, device="cuda",
                     pack_documents=a.doc_len > 0, eos_id=2, synthetic_doc_len=a.doc_len, graph=a.graph)
    tr = Trainer(tc)
    info = tr.info
    dev = tr.device

    def sync():
        torch.cuda.synchronize(dev)

    for _ in range(a.warmup):
        tr.train_step(tc.lr)
    sync()
    pdist.barrier(info)
    sync()
    _mark("push")  # roctx range "ftc_timed" (rocprofv3 --marker-trace; tools/kstats_md.py filters on it)
    t0 = time.perf_counter()
    last = None
    for _ in range(a.steps):
        last = tr.train_step(tc.lr)
    sync()
    pdist.barrier(info)
    sync()
    elapsed = time.perf_counter() - t0
    _mark("pop")
    elapsed = pdist.all_reduce_max(elapsed, info)
    loss = float(last.float().item()) if last is not None else float("nan")

    n = info.world_size
    tokens = a.batch_size * a.seq_len * n * a.steps
    value = tokens / elapsed
    ms = elapsed / a.steps * 1000
    flops_tok = tr.cfg.flops_per_token(a.seq_len, lora=a.method != "full")
    if a.profile_steps:
        from torch.profiler import ProfilerActivity, profile

        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(a.profile_steps):
                tr.train_step(tc.lr)
            sync()
        if info.is_main:
            os.makedirs("gpurun_out", exist_ok=True)
            with open("gpurun_out/torch_profile.txt", "w") as f:
                f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60))
    if info.is_main:
        from finetune_controller_amd.ops import _backend

        out = {
            "metric": BASELINE_METRIC,
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": n,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (uniform random token ids; random-init weights)",
            "config": {
                "model": "llama3-8b" if a.model == "llama3-8b" else a.model,
                "method": a.method,
                "lora": {"r": a.lora_r, "alpha": 2 * a.lora_r, "targets": "all-linear"} if a.method != "full" else None,
                "global_batch": a.batch_size * n,
                "micro_batch_per_gpu": a.batch_size,
                "seq_len": a.seq_len,
                "tokens_per_step": a.batch_size * a.seq_len * n,
                "parallelism": f"dp{n}" + ("-zero1" if a.zero_stage and n > 1 else ""),
                "kernels": _backend.kernel_mode(),
                "comm_engine": a.comm_engine,
                "zero_stage": a.zero_stage,
                **({"packed_doc_len": a.doc_len} if a.doc_len else {}),
                **({"hipgraph": True} if tr.graph_ok() else {}),
            },
            "loss": round(loss, 4),
            "model_tflops_per_gpu": round(value * flops_tok / n / 1e12, 1),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1),
        }
        print(json.dumps(out), flush=True)
    tr.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
