"""LoRA adapters over packed projections, with PEFT-compatible export.

A decoder layer owns four packed projections (SURVEY.md §2.3 K5 shapes):

==========  ===========================  ========================
projection  packed segments (rows)       PEFT module names
==========  ===========================  ========================
``qkv``     q (H*D), k (KV*D), v (KV*D)  q_proj, k_proj, v_proj
``o``       o (d)                        o_proj
``gu``      gate (F), up (F)             gate_proj, up_proj
``down``    down (d)                     down_proj
==========  ===========================  ========================

For each projection a :class:`LoRAPair` holds ``A = [A_s1; A_s2; ...]`` (one stacked GEMM) and a
block-diagonal ``B`` whose diagonal blocks are the per-segment ``B_s`` (one GEMM with K = n*r).
Segments not targeted get no rank slice at all.  ``export_peft`` writes the per-module
``lora_A`` / ``lora_B`` tensors under the PEFT key names, so adapters trained here load into
PEFT/transformers and vice versa.
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field

import torch
import torch.nn as nn

ALL_LINEAR = ["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj"]


@dataclass
class LoRAConfig:
    r: int = 16
    alpha: float = 32.0
    dropout: float = 0.0
    target_modules: list[str] = field(default_factory=lambda: list(ALL_LINEAR))
    use_rslora: bool = False  # rank-stabilised scaling alpha / sqrt(r) (PEFT ``use_rslora``)

    def __post_init__(self):
        bad = [t for t in self.target_modules if t not in ALL_LINEAR]
        if bad or not self.target_modules:
            raise ValueError(f"unknown LoRA target module(s) {bad or self.target_modules}: choose from {ALL_LINEAR}")

    @property
    def scale(self) -> float:
        return self.alpha / (self.r ** 0.5 if self.use_rslora else self.r)

    def to_peft(self, base_model: str) -> dict:
        return {"peft_type": "LORA", "task_type": "CAUSAL_LM", "r": self.r, "lora_alpha": self.alpha,
                "lora_dropout": self.dropout, "target_modules": list(self.target_modules), "bias": "none",
                "base_model_name_or_path": base_model, "fan_in_fan_out": False, "inference_mode": False,
                "use_rslora": self.use_rslora}

    def to_dict(self):
        return asdict(self)


class LoRAPair(nn.Module):
    """Stacked A / block-diagonal B for one packed projection."""

    def __init__(self, in_features: int, segments: list[tuple[str, int]], targets: list[str], cfg: LoRAConfig,
                 device=None, dtype=torch.bfloat16):
        super().__init__()
        self.r, self.scale = cfg.r, cfg.scale
        self.dropout = float(cfg.dropout)
        self.in_features = in_features
        self.names: list[str] = []
        blocks, row = [], 0
        col = 0
        for name, rows in segments:
            if name in targets:
                blocks.append((row, row + rows, col, col + cfg.r))
                self.names.append(name)
                col += cfg.r
            row += rows
        self.out_features = row
        self.rank_total = col
        self.blocks = blocks if len(blocks) > 1 or (blocks and (blocks[0][0] != 0 or blocks[0][1] != row)) else None
        self.segments = segments
        self.A = nn.Parameter(torch.empty(col, in_features, device=device, dtype=dtype))
        self.B = nn.Parameter(torch.zeros(row, col, device=device, dtype=dtype))
        self.reset_parameters()

    @property
    def active(self) -> bool:
        return self.rank_total > 0

    def reset_parameters(self):
        # PEFT default: kaiming-uniform(a=sqrt(5)) A, zero B -> the adapter starts as the identity
        with torch.no_grad():
            bound = 1.0 / math.sqrt(self.in_features)
            self.A.uniform_(-bound, bound)
            self.B.zero_()

    def segment_tensors(self):
        """Yield (segment_name, A_s [r,in], B_s [rows_s, r])."""
        i = 0
        row = 0
        for name, rows in self.segments:
            if name in self.names:
                yield name, self.A[i * self.r:(i + 1) * self.r], self.B[row:row + rows, i * self.r:(i + 1) * self.r]
                i += 1
            row += rows

    @torch.no_grad()
    def load_segment(self, name: str, A_s: torch.Tensor, B_s: torch.Tensor):
        i = self.names.index(name)
        row = 0
        for n, rows in self.segments:
            if n == name:
                break
            row += rows
        self.A[i * self.r:(i + 1) * self.r].copy_(A_s)
        self.B[row:row + B_s.shape[0], i * self.r:(i + 1) * self.r].copy_(B_s)

    def zero_segment(self, name: str):
        """Segment ``name`` contributes nothing (B = 0; A kept): a slot an adapter does not train."""
        i = self.names.index(name)
        row = 0
        for n, rows in self.segments:
            if n == name:
                self.B[row:row + rows, i * self.r:(i + 1) * self.r].zero_()
                return
            row += rows


def make_pairs(layer_shapes: dict[str, tuple[int, list[tuple[str, int]]]], cfg: LoRAConfig, device=None,
               dtype=torch.bfloat16) -> nn.ModuleDict:
    pairs = nn.ModuleDict()
    for proj, (in_f, segs) in layer_shapes.items():
        p = LoRAPair(in_f, segs, cfg.target_modules, cfg, device=device, dtype=dtype)
        if p.active:
            pairs[proj] = p
    return pairs


@torch.no_grad()
def merge_pair_into(W: torch.Tensor, pair: LoRAPair, sign: float = 1.0):
    """W += sign * scale * B A (per segment; HIP kernel K6 on GPU)."""
    from ..ops._backend import ext, use_hip

    row = 0
    i = 0
    for name, rows in pair.segments:
        if name in pair.names:
            A_s = pair.A[i * pair.r:(i + 1) * pair.r].to(W.dtype).contiguous()
            B_s = pair.B[row:row + rows, i * pair.r:(i + 1) * pair.r].to(W.dtype).contiguous()
            Wv = W[row:row + rows]
            if use_hip(W) and W.dtype == torch.bfloat16:
                if Wv.is_contiguous():
                    ext().lora_merge_(Wv, A_s, B_s, sign * pair.scale, 0)
                else:  # column view of an augmented weight buffer (ops/linear.py)
                    Wc = Wv.contiguous()
                    ext().lora_merge_(Wc, A_s, B_s, sign * pair.scale, 0)
                    Wv.copy_(Wc)
            else:
                Wv.add_((B_s.float() @ A_s.float()).to(W.dtype), alpha=sign * pair.scale)
            i += 1
        row += rows
