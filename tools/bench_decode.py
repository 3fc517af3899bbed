#!/usr/bin/env python3
"""Generation throughput with the KV cache: B prompts of P tokens prefilled, then N decode steps of
one token per sequence (``models.generate``).  Random-init weights, synthetic prompts; prints one
JSON line with prefill and decode rates."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--prompt-len", type=int, default=1024)
    ap.add_argument("--new-tokens", type=int, default=64)
    ap.add_argument("--lora", action="store_true", help="live LoRA r=16 adapters (augmented GEMMs)")
    ap.add_argument("--eager", action="store_true", help="decode steps issued from Python (no hipGraph)")
    a = ap.parse_args()
    from finetune_controller_amd import ops
    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import get_config
    from finetune_controller_amd.models.generate import DecodeStep

    cfg = get_config(a.model)
    dev = torch.device("cuda")
    m = build_model(cfg, LoRAConfig(r=16, alpha=32) if a.lora else None, device=dev, dtype=torch.bfloat16)
    m.init_weights(seed=0)
    m.eval()
    g = torch.Generator().manual_seed(0)
    prompts = torch.randint(3, cfg.vocab_size, (a.batch, a.prompt_len), generator=g).to(dev)
    B, P, N = a.batch, a.prompt_len, a.new_tokens
    cache = ops.KVCache(len(m.layers), B, P + N + 1, cfg.n_kv_heads, cfg.head_dim, dev)
    with torch.no_grad():
        # warm-up pass on a small cache (hipBLASLt heuristics, kernel loads)
        wc = ops.KVCache(len(m.layers), B, 64, cfg.n_kv_heads, cfg.head_dim, dev)
        for b in range(B):
            wc.row = b
            m.hidden(prompts[b:b + 1, :32], kv_cache=wc)
            wc.finish_prefill(b, 32)
        pos = wc.begin_decode()
        m.hidden(prompts[:, :1], positions=pos, kv_cache=wc)
        wc.end_decode()
        wc.decoding = False
        del wc
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b in range(B):
            cache.row = b
            m.hidden(prompts[b:b + 1], kv_cache=cache)
            cache.finish_prefill(b, P)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step = DecodeStep(m, cache, B, graph=not a.eager)
        tok = prompts[:, -1]
        for _ in range(N):
            tok = step(tok).argmax(-1)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    print(json.dumps({"model": a.model, "lora": a.lora, "hipgraph": not a.eager, "batch": B, "prompt_len": P, "new_tokens": N,
                      "prefill_tok_s": round(B * P / (t1 - t0), 1), "decode_tok_s": round(B * N / (t2 - t1), 1),
                      "decode_ms_per_step": round((t2 - t1) / N * 1000, 2),
                      "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
