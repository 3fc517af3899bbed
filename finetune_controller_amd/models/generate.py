"""Text generation with a KV cache for the Llama / Mistral trunk (checking a fine-tuned model, or
serving it from a promoted artifact).

``generate(model, prompts, ...)``: each prompt is prefilled on its own (flash attention over the
prompt, K/V rows written into the cache), then all sequences decode together -- one token per
sequence per step through ``ops.decode_attention`` (split-K decode kernel on MI355X).  LoRA adapters
stay live in the augmented GEMMs (``checkpoint.save_full`` exports them merged).  Greedy by default; ``temperature`` / ``top_p`` sample with a seeded
generator.  Lengths are tracked on the host so the loop never reads device memory except for the
sampled tokens themselves.

On MI355X the decode step (every layer's GEMMs, RoPE at the cache position, the K/V append, the
decode-attention kernel and the lm_head GEMM) is captured once in a hipGraph and replayed per token:
a decode step is a few ms of GPU work spread over ~20 launches per layer, so issuing it from Python
would leave the GPU idle most of the time (``graph=False`` keeps the eager loop).
"""
from __future__ import annotations

import torch

from .. import ops


@torch.no_grad()
def _sample(logits: torch.Tensor, temperature: float, top_p: float, gen: torch.Generator | None) -> torch.Tensor:
    if temperature <= 0.0:
        return logits.argmax(-1)
    probs = torch.softmax(logits.float() / temperature, -1)
    if 0.0 < top_p < 1.0:
        sp, si = probs.sort(-1, descending=True)
        keep = sp.cumsum(-1) - sp < top_p  # the smallest prefix whose mass reaches top_p
        sp = sp * keep
        pick = torch.multinomial(sp / sp.sum(-1, keepdim=True), 1, generator=gen)
        return si.gather(-1, pick).squeeze(-1)
    return torch.multinomial(probs, 1, generator=gen).squeeze(-1)


@torch.no_grad()
def generate(model, prompts: list[list[int]], max_new_tokens: int = 32, temperature: float = 0.0, top_p: float = 1.0,
             eos_id: int | None = None, seed: int = 0, graph: bool | None = None) -> list[list[int]]:
    """Continue every prompt (a list of token ids) by up to ``max_new_tokens`` tokens; returns the
    generated ids per prompt (stopping after ``eos_id``)."""
    if not hasattr(model, "layers") or not hasattr(model, "rope"):
        raise NotImplementedError("generate(): Llama / Mistral trunk models only")
    was = model.training
    model.eval()
    cfg = model.cfg
    dev = model.embed.device
    B = len(prompts)
    max_len = max(len(p) for p in prompts) + max_new_tokens
    if max_len > model.rope.max_pos:
        raise ValueError(f"prompt + new tokens = {max_len} exceeds the model's {model.rope.max_pos} positions")
    cache = ops.KVCache(len(model.layers), B, max_len, cfg.n_kv_heads, cfg.head_dim, dev, model.embed.dtype)
    gen = torch.Generator(device=dev).manual_seed(seed) if temperature > 0 else None
    try:
        # prefill, one prompt at a time (prompts differ in length)
        nxt = []
        for b, p in enumerate(prompts):
            if not p:
                raise ValueError("empty prompt")
            cache.row = b
            ids = torch.tensor([p], dtype=torch.long, device=dev)
            x = model.hidden(ids, kv_cache=cache)
            logits = x[-1:] @ model.lm_head.t()
            nxt.append(_sample(logits, temperature, top_p, gen))
            cache.finish_prefill(b, len(p))
        tok = torch.cat(nxt)  # [B]
        out = [[] for _ in range(B)]
        done = [False] * B
        step_fn = DecodeStep(model, cache, B, graph)
        for step in range(max_new_tokens):
            host = tok.tolist()
            for b in range(B):
                if not done[b]:
                    out[b].append(host[b])
                    done[b] = eos_id is not None and host[b] == eos_id
            if all(done) or step == max_new_tokens - 1:
                break
            tok = _sample(step_fn(tok), temperature, top_p, gen)
        return out
    finally:
        cache.decoding = False
        model.train(was)


class DecodeStep:
    """tokens [B] -> next-token logits [B, vocab], appending to the cache.  The first call runs eagerly
    (warms hipBLASLt and the caches); on a GPU the second is captured in a hipGraph and every call from
    then on replays it with the new tokens copied into its static input."""

    def __init__(self, model, cache, B: int, graph: bool | None = None):
        self.model, self.cache, self.B = model, cache, B
        dev = cache.k.device
        self.use_graph = (dev.type == "cuda") if graph is None else (graph and dev.type == "cuda")
        self.calls = 0
        self.g = None

    def _body(self, tok):
        cache, model = self.cache, self.model
        pos = cache.begin_decode()
        x = model.hidden(tok.view(self.B, 1), positions=pos, kv_cache=cache)
        cache.lens += 1
        return x @ model.lm_head.t()

    def __call__(self, tok: torch.Tensor) -> torch.Tensor:
        cache = self.cache
        self.calls += 1
        if not self.use_graph or self.calls == 1:
            logits = self._body(tok)
        elif self.g is None:
            cache.graph_mode = True
            self.tok = tok.view(self.B).clone()
            torch.cuda.synchronize()
            self.g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g):
                self.logits = self._body(self.tok)
            self.g.replay()  # the capture ran nothing
            logits = self.logits
        else:
            self.tok.copy_(tok.view(self.B))
            self.g.replay()
            logits = self.logits
        cache.decoding = False
        cache.host_lens = [n + 1 for n in cache.host_lens]
        return logits


def peft_targets(tm) -> list[str]:
    """A PEFT ``target_modules`` entry as this model's projection names: ``"all-linear"``, a list, or one
    name / regex-like string; modules this model has no LoRA slot for (an adapter from another tool that
    also targets ``lm_head``, say) are dropped with a warning."""
    import sys

    from .lora import ALL_LINEAR

    if tm is None or tm == "all-linear":
        return list(ALL_LINEAR)
    names = [tm] if isinstance(tm, str) else list(tm)
    if len(names) == 1 and names[0] not in ALL_LINEAR:
        names = [t for t in ALL_LINEAR if t in str(names[0])] or names  # e.g. ".*(q_proj|v_proj)$"
    kept = [t for t in names if t in ALL_LINEAR]
    dropped = [t for t in names if t not in ALL_LINEAR]
    if dropped:
        print(f"[generate] adapter targets without a LoRA slot here, ignored: {dropped}", file=sys.stderr)
    if not kept:
        raise ValueError(f"adapter targets {tm!r} name none of {ALL_LINEAR}")
    return kept


def main(argv=None) -> int:
    """``python -m finetune_controller_amd.models.generate --model llama3-8b [--init-from HF_DIR]
    [--adapter ADAPTER_DIR] --prompt "..."``: continue prompts with a (fine-tuned) model."""
    import argparse
    import os

    from ..train.data import Tokenizer
    from . import LoRAConfig, build_model
    from . import checkpoint as ckpt
    from .config import get_config

    ap = argparse.ArgumentParser(prog="ftc-generate")
    ap.add_argument("--model", default="llama3-8b", help="preset name or HF config.json")
    ap.add_argument("--init-from", default="", help="HF safetensors checkpoint dir")
    ap.add_argument("--adapter", default="", help="PEFT adapter dir (adapter_config.json + weights)")
    ap.add_argument("--tokenizer", default="", help="dir with tokenizer.json (default: byte-level)")
    ap.add_argument("--prompt", action="append", required=True)
    ap.add_argument("--max-new-tokens", type=int, default=64)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--top-p", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args(argv)
    cfg = get_config(a.model)
    dev = torch.device("cuda" if torch.cuda.device_count() > 0 and torch.cuda.is_available() else "cpu")
    lora = None
    if a.adapter:
        import json

        with open(os.path.join(a.adapter, "adapter_config.json")) as f:
            ac = json.load(f)
        lora = LoRAConfig(r=ac["r"], alpha=ac["lora_alpha"], target_modules=peft_targets(ac.get("target_modules")),
                          use_rslora=bool(ac.get("use_rslora", False)))
    m = build_model(cfg, lora, device=dev, dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32)
    if a.init_from:
        ckpt.load_hf_checkpoint(m, a.init_from)
    else:
        m.init_weights(seed=a.seed)
    if a.adapter:
        ckpt.load_adapter(m, a.adapter)
    tok = Tokenizer(a.tokenizer or None, cfg.vocab_size)
    prompts = [tok.encode(p) for p in a.prompt]
    outs = generate(m, prompts, a.max_new_tokens, a.temperature, a.top_p, eos_id=tok.eos, seed=a.seed)
    for p, o in zip(a.prompt, outs):
        text = tok.tk.decode(o) if tok.tk is not None else bytes(max(0, t - 3) for t in o if 3 <= t < 259).decode(
            "utf-8", errors="replace")
        print(f"{p}{text}", flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
