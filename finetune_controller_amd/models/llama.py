"""Llama-3 / Mistral decoder (one trunk; Mistral = sliding-window attention + its own vocab/RoPE).

MI355X-first layout decisions (not a port of any reference module -- the reference has no model
code):

* **Packed frozen weights.** q/k/v live in one ``Wqkv [(H+2KV)*D, d]`` and gate/up in one
  ``Wgu [2F, d]``: two GEMMs per layer fewer, each larger (better MFMA occupancy on 256 CUs), and
  the RoPE / attention / SwiGLU kernels read the packed outputs in place.
* **Residual add fused into every norm** (``add_rms_norm``): the residual stream ``h`` and the
  sub-block output are combined by the norm kernel itself.
* **No activation checkpointing by default**: with 288 GB of HBM a frozen-base LoRA step keeps all
  activations of 16k tokens of Llama-3-8B resident (≈4.2 MB/token), saving the 33 % recompute.
  ``checkpoint_layers`` is available for longer sequences / full FT.
* **Loss through the chunked fused linear+CE** (never [tokens, vocab] fp32 logits).

Weight names map 1:1 onto Hugging Face ``LlamaForCausalLM`` / ``MistralForCausalLM`` (see
``checkpoint.py``), so random-init benchmarks and real checkpoints use the same module.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.utils.checkpoint import checkpoint

from .. import ops
from .config import ModelConfig
from ..ops.linear import AugWeight, LoRATail, TailOperands
from ..ops.mlp import AugProj, NF4Proj, fused_mlp_supported, lora_mlp
from .lora import LoRAConfig, make_pairs


class LlamaLayer(nn.Module):
    def __init__(self, cfg: ModelConfig, lora: LoRAConfig | None, device=None, dtype=torch.bfloat16):
        super().__init__()
        d, D, H, KV, Fd = cfg.dim, cfg.head_dim, cfg.n_heads, cfg.n_kv_heads, cfg.ffn_dim
        self.cfg = cfg
        kw = dict(device=device, dtype=dtype)
        self.attn_norm = nn.Parameter(torch.ones(d, **kw))
        self.wqkv = nn.Parameter(torch.empty((H + 2 * KV) * D, d, **kw))
        self.wo = nn.Parameter(torch.empty(d, H * D, **kw))
        self.mlp_norm = nn.Parameter(torch.ones(d, **kw))
        self.wgu = nn.Parameter(torch.empty(2 * Fd, d, **kw))
        self.wdown = nn.Parameter(torch.empty(d, Fd, **kw))
        self.shapes = {
            "qkv": (d, [("q_proj", H * D), ("k_proj", KV * D), ("v_proj", KV * D)]),
            "o": (H * D, [("o_proj", d)]),
            "gu": (d, [("gate_proj", Fd), ("up_proj", Fd)]),
            "down": (Fd, [("down_proj", d)]),
        }
        self.lora = make_pairs(self.shapes, lora, device=device, dtype=dtype) if lora else nn.ModuleDict()
        self.qweights: dict[str, object] = {}  # QLoRA: proj -> NF4Weight (replaces the bf16 Parameter)
        self.qtails: dict[str, TailOperands] = {}  # QLoRA: LoRA tail operands for fused producers
        # LoRA: the frozen base weight lives inside an augmented [N+R, K+R] buffer (ops.linear.AugWeight)
        # so the rank-r update rides along in the big GEMMs; the Parameter is a view of it
        self.aug: dict[str, AugWeight] = {}
        attr = {"qkv": "wqkv", "o": "wo", "gu": "wgu", "down": "wdown"}
        for name, pair in self.lora.items():
            R = pair.A.shape[0]
            if R > 0:
                W = getattr(self, attr[name])
                aw = AugWeight(W.shape[0], W.shape[1], R, device=device, dtype=dtype)
                setattr(self, attr[name], nn.Parameter(aw.W, requires_grad=W.requires_grad))
                self.aug[name] = aw

    def base_weight(self, proj: str):
        return {"qkv": self.wqkv, "o": self.wo, "gu": self.wgu, "down": self.wdown}[proj]

    def pad(self, name: str) -> int:
        """Spare columns the producer of this projection's input (and of its output gradient) adds."""
        if os.environ.get("FTC_LORA_AUG", "1") == "0":  # A/B switch: two-GEMM LoRA path
            return 0
        if name in self.qweights:  # QLoRA: the NF4 path augments its dequantised operand the same way
            pair = self.lora[name] if name in self.lora else None
            return -(-pair.A.shape[0] // AugWeight.TILE) * AugWeight.TILE if pair is not None else 0
        aw = self.aug.get(name)
        if aw is None or not aw.owns(self.base_weight(name)):
            return 0
        return aw.Rp

    def tail(self, name: str, pad: int):
        """LoRATail of an augmented projection (its producer kernel may form the rank-r tail product),
        or None where the consumer does not take the augmented path (LoRA dropout, no pad)."""
        if pad <= 0 or name not in self.lora:
            return None
        pair = self.lora[name]
        if self.training and pair.dropout > 0.0:
            return None
        if name in self.qweights:  # QLoRA: stand-alone tail operands next to the NF4 weight
            qt = self.qtails.get(name)
            if qt is None or qt.Rp != pad:
                N, K = self.qweights[name].shape
                qt = self.qtails[name] = TailOperands(N, K, pair.A.shape[0], pad, device=pair.A.device,
                                                      dtype=pair.A.dtype)
            return LoRATail(qt, pair.A, pair.B, pair.scale, pair.blocks)
        aw = self.aug.get(name)
        if aw is None:
            return None
        return LoRATail(aw, pair.A, pair.B, pair.scale, pair.blocks)

    def mlp_projs(self, p_gu: int, p_down: int):
        """(gate|up, down) projections for ops.mlp.lora_mlp: AugProj (bf16) or NF4Proj (QLoRA), or None."""
        if "gu" not in self.lora or "down" not in self.lora or p_gu <= 0 or p_down <= 0:
            return None
        out = []
        for name, pad in (("gu", p_gu), ("down", p_down)):
            pair = self.lora[name]
            if name in self.qweights:
                t = self.tail(name, pad)  # creates the TailOperands
                if t is None:
                    return None
                out.append(NF4Proj(self.qweights[name], self.qtails[name], pair))
            else:
                aw = self.aug.get(name)
                if aw is None or not aw.owns(self.base_weight(name)):
                    return None
                out.append(AugProj(aw, pair))
        return tuple(out)

    def proj(self, name: str, x: torch.Tensor, rope: tuple | None = None) -> torch.Tensor:
        pair = self.lora[name] if name in self.lora else None
        qw = self.qweights.get(name)
        if qw is not None:
            from ..ops.nf4 import qlora_linear

            return qlora_linear(x, qw, pair.A if pair else None, pair.B if pair else None,
                                pair.scale if pair else 1.0, pair.blocks if pair else None, pad=self.pad(name),
                                tails=self.qtails.get(name))
        W = self.base_weight(name)
        if pair is None:
            return ops.lora_linear(x, W)
        return ops.lora_linear(x, W, pair.A, pair.B, pair.scale, blocks=pair.blocks, aug=self.aug.get(name),
                               dropout=pair.dropout if self.training else 0.0, rope=rope)

    def forward(self, h, delta, rope: ops.RotaryTable, B: int, S: int, positions=None, docs=None, kv=None):
        cfg = self.cfg
        p_qkv, p_o, p_gu, p_down = (self.pad(n) for n in ("qkv", "o", "gu", "down"))
        # grad_pad: delta came from the previous layer's down projection (same LoRA shape in every layer;
        # a pad that is too small just falls back to the two-GEMM backward)
        h, x = ops.add_rms_norm(h, delta, self.attn_norm, cfg.norm_eps, pad=p_qkv, grad_pad=p_down)
        # RoPE inside the qkv projection (fused into the GEMM epilogue where the hand-written kernel runs
        # it) for the LoRA GPU path; elsewhere the separate in-place op
        rargs = rgrad = None
        hip_bf16 = ops.use_hip(x) and x.dtype == torch.bfloat16 and cfg.head_dim == 128 and x.dim() == 2
        if hip_bf16 and kv is None and getattr(self, "sp", None) is None:
            # full-sequence attention on this rank: the flash backward may take RoPE's inverse rotation
            cos, sin = rope.get(x.device)
            pos = positions.to(torch.int32).contiguous() if positions is not None else None
            rgrad = ops.RopeGrad(cos, sin, pos)
        if hip_bf16 and "qkv" in self.lora and "qkv" not in self.qweights:
            cos, sin = rope.get(x.device)
            pos = positions.to(torch.int32).contiguous() if positions is not None else None
            rargs = (cos, sin, pos, S, cfg.n_heads + cfg.n_kv_heads, cfg.head_dim, rgrad)
        qkv = self.proj("qkv", x, rope=rargs)
        if rargs is None:
            qkv = ops.apply_rope_packed(qkv, rope, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, S, positions,
                                        handoff=rgrad)
        if kv is not None and kv[0].decoding:  # generation: one new token per sequence vs its cache
            cache, li = kv
            a = ops.decode_attention(qkv, cache.k[li], cache.v[li], cache.lens_next, cache.attend_len(),
                                     cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, window=cfg.sliding_window)
        else:
            if kv is not None:  # prefill: keep this prompt's K/V rows
                kv[0].store(kv[1], qkv, cfg.n_heads, S)
            sp = getattr(self, "sp", None)
            if sp is not None and kv is None:  # Ulysses: heads <-> tokens all-to-all around full-sequence attention
                from ..parallel.sequence import sp_attention

                a = sp_attention(qkv, B, S, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, cfg.sliding_window, sp)
            else:
                a = ops.attention_packed(qkv, B, S, cfg.n_heads, cfg.n_kv_heads, cfg.head_dim, True,
                                         cfg.sliding_window, out_pad=p_o, grad_pad=p_qkv, docs=docs,
                                         rope_grad=rgrad)
        o = self.proj("o", a)
        h, x = ops.add_rms_norm(h, o, self.mlp_norm, cfg.norm_eps, pad=p_gu, grad_pad=p_o)
        mlp = self.mlp_projs(p_gu, p_down)
        if mlp is not None and fused_mlp_supported(x, mlp[0], mlp[1], self.lora["gu"], self.lora["down"], p_gu,
                                                   p_down, self.training):
            # the whole LoRA MLP as one autograd function: SwiGLU backward also forms dB_gu / dA_down
            return h, lora_mlp(x, mlp[0], mlp[1])
        gu = self.proj("gu", x)
        act = ops.swiglu(gu, out_pad=p_down, grad_pad=p_gu, fwd_tail=self.tail("down", p_down),
                         bwd_tail=self.tail("gu", p_gu))
        return h, self.proj("down", act)


class LlamaForCausalLM(nn.Module):
    def __init__(self, cfg: ModelConfig, lora: LoRAConfig | None = None, device=None, dtype=torch.bfloat16,
                 checkpoint_layers: bool = False):
        super().__init__()
        self.cfg, self.lora_cfg = cfg, lora
        kw = dict(device=device, dtype=dtype)
        self.embed = nn.Parameter(torch.empty(cfg.vocab_size, cfg.dim, **kw))
        self.layers = nn.ModuleList([LlamaLayer(cfg, lora, device, dtype) for _ in range(cfg.n_layers)])
        self.final_norm = nn.Parameter(torch.ones(cfg.dim, **kw))
        self.lm_head = self.embed if cfg.tie_embeddings else nn.Parameter(torch.empty(cfg.vocab_size, cfg.dim, **kw))
        self.rope = ops.RotaryTable(cfg.head_dim, cfg.max_seq_len, cfg.rope_theta, cfg.rope_scaling)
        self.checkpoint_layers = checkpoint_layers
        self.ce_chunk_rows = 4096
        # set by the trainer when the optimizer update overlaps the next forward (FlatAdamW.enable_overlap):
        # called with the stage index before the stage's parameters are read
        self.param_gate = None
        self.sp = None  # parallel.sequence.SeqGroup: this rank holds 1/P of every sequence (set_sequence_parallel)

    def set_sequence_parallel(self, sp):
        """Ulysses sequence parallelism (parallel/sequence.py): inputs are this rank's contiguous 1/P of
        each sequence, RoPE uses global positions, attention runs over the whole sequence on H/P heads."""
        self.sp = sp
        for layer in self.layers:
            layer.sp = sp

    def param_stages(self) -> list[list[nn.Parameter]]:
        """Parameters in forward order of first use: [embed], [layer 0], ..., [layer L-1], [final norm,
        lm_head] -- the stages of ``param_gate``."""
        stages = [[self.embed]] + [list(layer.parameters()) for layer in self.layers] + [[self.final_norm]]
        if self.lm_head is not self.embed:
            stages[-1].append(self.lm_head)
        return stages

    @torch.no_grad()
    def init_weights(self, seed: int = 0, std: float = 0.02):
        """Random init (synthetic benchmarks). Generated on the parameters' own device."""
        g = torch.Generator(device=self.embed.device).manual_seed(seed)
        out_std = std / math.sqrt(2 * self.cfg.n_layers)
        for name, p in self.named_parameters():
            if ".lora." in name:
                continue
            if p.dim() == 1:
                p.fill_(1.0)
            elif name.endswith("wo") or name.endswith("wdown"):
                p.normal_(0.0, out_std, generator=g)
            else:
                p.normal_(0.0, std, generator=g)
        for layer in self.layers:
            for pair in layer.lora.values():
                pair.reset_parameters()
        self.invalidate_transposed()

    def invalidate_transposed(self):
        """Base weights were rewritten: drop the transposed backward copies (ops.linear TN layout)."""
        from ..ops.linear import frozen_t

        for layer in self.layers:
            for aw in layer.aug.values():
                aw.invalidate()
        frozen_t.clear()

    def freeze_base(self):
        """LoRA/QLoRA: only adapter parameters train."""
        for name, p in self.named_parameters():
            p.requires_grad_(".lora." in name)

    def hidden(self, input_ids: torch.Tensor, positions=None, segments=None, kv_cache=None) -> torch.Tensor:
        """``segments`` (``ops.Segments``): packed documents -- RoPE positions restart and attention
        stays inside each document."""
        B, S = input_ids.shape
        if segments is not None:
            positions = segments.positions
        gate = self.param_gate
        if gate is not None:
            gate(0)
        h = F.embedding(input_ids.reshape(-1), self.embed)
        delta = None
        for li, layer in enumerate(self.layers):
            if gate is not None:
                gate(li + 1)
            if self.checkpoint_layers and self.training and torch.is_grad_enabled():
                h, delta = checkpoint(layer, h, delta, self.rope, B, S, positions, segments, use_reentrant=False)
            else:
                h, delta = layer(h, delta, self.rope, B, S, positions, segments,
                                 (kv_cache, li) if kv_cache is not None else None)
        gp = self.layers[-1].pad("down") if len(self.layers) else 0
        if gate is not None:
            gate(len(self.layers) + 1)
        _, x = ops.add_rms_norm(h, delta, self.final_norm, self.cfg.norm_eps, grad_pad=gp)
        return x

    def forward(self, input_ids: torch.Tensor, labels: torch.Tensor | None = None, positions=None,
                n_valid: int | None = None, segments=None):
        B, S = input_ids.shape
        if self.sp is not None:  # S = this rank's 1/P of each sequence (attention pads the full one itself)
            if segments is not None:
                raise ValueError("packed documents are not supported with sequence parallelism")
            if positions is None:
                positions = self.sp.positions(B, S, input_ids.device)
            x = self.hidden(input_ids, positions, None)
            if labels is None:
                return x @ self.lm_head.t()
            return ops.fused_linear_cross_entropy(x, self.lm_head, labels, self.ce_chunk_rows, -100, n_valid)
        Sp = ops.model_tile_len(S, self.cfg.head_dim, ops.use_hip(self.embed), self.embed.dtype, self.cfg.max_seq_len)
        if Sp != S:  # GPU, S off the flash tile: run the whole model tile-aligned (ops.attention.model_tile_len)
            input_ids, labels, positions, segments = ops.pad_batch_to(Sp, input_ids, labels, positions, segments)
        x = self.hidden(input_ids, positions, segments)
        if labels is None:
            logits = x @ self.lm_head.t()
            return logits if Sp == S else logits.view(B, Sp, -1)[:, :S].reshape(B * S, -1)
        return ops.fused_linear_cross_entropy(x, self.lm_head, labels, self.ce_chunk_rows, -100, n_valid)
