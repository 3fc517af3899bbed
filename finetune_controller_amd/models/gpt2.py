"""GPT-2 (small) -- the BASELINE.json plumbing config ("GPT-2-small full fine-tune PyTorchJob,
1 CPU worker via local Kueue").  LayerNorm + GELU(tanh) + learned positions, tied lm_head.

Runs on CPU for the FakeCluster e2e job and on GPU with the same packed-qkv attention op as the
Llama trunk (H = KV).  Parameter names map onto HF ``GPT2LMHeadModel`` in ``checkpoint.py``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint

from .. import ops
from .config import ModelConfig
from .lora import LoRAConfig, make_pairs


class GPT2Block(nn.Module):
    def __init__(self, cfg: ModelConfig, lora: LoRAConfig | None, device=None, dtype=torch.float32):
        super().__init__()
        d, Fd = cfg.dim, cfg.ffn_dim
        kw = dict(device=device, dtype=dtype)
        self.cfg = cfg
        self.ln1_w = nn.Parameter(torch.ones(d, **kw))
        self.ln1_b = nn.Parameter(torch.zeros(d, **kw))
        self.attn_w = nn.Parameter(torch.empty(3 * d, d, **kw))
        self.attn_b = nn.Parameter(torch.zeros(3 * d, **kw))
        self.proj_w = nn.Parameter(torch.empty(d, d, **kw))
        self.proj_b = nn.Parameter(torch.zeros(d, **kw))
        self.ln2_w = nn.Parameter(torch.ones(d, **kw))
        self.ln2_b = nn.Parameter(torch.zeros(d, **kw))
        self.fc_w = nn.Parameter(torch.empty(Fd, d, **kw))
        self.fc_b = nn.Parameter(torch.zeros(Fd, **kw))
        self.out_w = nn.Parameter(torch.empty(d, Fd, **kw))
        self.out_b = nn.Parameter(torch.zeros(d, **kw))
        shapes = {"qkv": (d, [("q_proj", d), ("k_proj", d), ("v_proj", d)]), "o": (d, [("o_proj", d)]),
                  "gu": (d, [("up_proj", Fd)]), "down": (Fd, [("down_proj", d)])}
        self.lora = make_pairs(shapes, lora, device=device, dtype=dtype) if lora else nn.ModuleDict()

    def _lin(self, name, x, W, b):
        p = self.lora[name] if name in self.lora else None
        if p is None:
            return ops.lora_linear(x, W, bias=b)
        return ops.lora_linear(x, W, p.A, p.B, p.scale, bias=b, blocks=p.blocks,
                               dropout=p.dropout if self.training else 0.0)

    def forward(self, h, B, S, docs=None):
        cfg = self.cfg
        x = ops.layer_norm(h, self.ln1_w, self.ln1_b, cfg.norm_eps)
        qkv = self._lin("qkv", x, self.attn_w, self.attn_b)
        a = ops.attention_packed(qkv, B, S, cfg.n_heads, cfg.n_heads, cfg.head_dim, True, 0, docs=docs)
        h = h + self._lin("o", a, self.proj_w, self.proj_b)
        x = ops.layer_norm(h, self.ln2_w, self.ln2_b, cfg.norm_eps)
        x = ops.gelu_tanh(self._lin("gu", x, self.fc_w, self.fc_b))
        return h + self._lin("down", x, self.out_w, self.out_b)


class GPT2ForCausalLM(nn.Module):
    def __init__(self, cfg: ModelConfig, lora: LoRAConfig | None = None, device=None, dtype=torch.float32,
                 checkpoint_layers: bool = False):
        super().__init__()
        self.cfg, self.lora_cfg = cfg, lora
        kw = dict(device=device, dtype=dtype)
        self.wte = nn.Parameter(torch.empty(cfg.vocab_size, cfg.dim, **kw))
        self.wpe = nn.Parameter(torch.empty(cfg.max_seq_len, cfg.dim, **kw))
        self.blocks = nn.ModuleList([GPT2Block(cfg, lora, device, dtype) for _ in range(cfg.n_layers)])
        self.lnf_w = nn.Parameter(torch.ones(cfg.dim, **kw))
        self.lnf_b = nn.Parameter(torch.zeros(cfg.dim, **kw))
        self.checkpoint_layers = checkpoint_layers
        self.ce_chunk_rows = 4096

    @property
    def lm_head(self):
        return self.wte

    @torch.no_grad()
    def init_weights(self, seed: int = 0, std: float = 0.02):
        g = torch.Generator(device=self.wte.device).manual_seed(seed)
        for name, p in self.named_parameters():
            if ".lora." in name:
                continue
            if name.endswith("_b"):
                p.zero_()
            elif p.dim() == 1:
                p.fill_(1.0)
            else:
                p.normal_(0.0, std if name != "wpe" else 0.01, generator=g)
        for b in self.blocks:
            for pair in b.lora.values():
                pair.reset_parameters()

    def freeze_base(self):
        for name, p in self.named_parameters():
            p.requires_grad_(".lora." in name)

    def hidden(self, input_ids, positions=None, segments=None):
        B, S = input_ids.shape
        if segments is not None:  # packed documents: positions restart per document
            pos = segments.positions.view(B, S).long()
            h = (self.wte[input_ids] + self.wpe[pos]).reshape(B * S, -1)
        else:
            pos = torch.arange(S, device=input_ids.device) if positions is None else positions.long()
            h = (self.wte[input_ids] + self.wpe[pos].view(-1, S, self.wpe.shape[1])).reshape(B * S, -1)
        for blk in self.blocks:
            if self.checkpoint_layers and self.training and torch.is_grad_enabled():
                h = checkpoint(blk, h, B, S, segments, use_reentrant=False)
            else:
                h = blk(h, B, S, segments)
        return ops.layer_norm(h, self.lnf_w, self.lnf_b, self.cfg.norm_eps)

    def forward(self, input_ids, labels=None, positions=None, n_valid=None, segments=None):
        B, S = input_ids.shape
        Sp = ops.model_tile_len(S, self.cfg.head_dim, ops.use_hip(self.wte), self.wte.dtype, self.cfg.max_seq_len)
        if Sp != S:  # GPU, S off the flash tile: run tile-aligned (ops.attention.model_tile_len)
            input_ids, labels, positions, segments = ops.pad_batch_to(Sp, input_ids, labels, positions, segments)
        x = self.hidden(input_ids, positions, segments)
        if labels is None:
            logits = x @ self.wte.t()
            return logits if Sp == S else logits.view(B, Sp, -1)[:, :S].reshape(B * S, -1)
        return ops.fused_linear_cross_entropy(x, self.wte, labels, self.ce_chunk_rows, -100, n_valid)


def build_model(cfg: ModelConfig, lora: LoRAConfig | None = None, device=None, dtype=None,
                checkpoint_layers: bool = False):
    if cfg.family == "gpt2":
        return GPT2ForCausalLM(cfg, lora, device, dtype or torch.float32, checkpoint_layers)
    from .llama import LlamaForCausalLM

    return LlamaForCausalLM(cfg, lora, device, dtype or torch.bfloat16, checkpoint_layers)
