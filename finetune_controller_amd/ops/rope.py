"""Rotary position embedding applied IN PLACE to the packed qkv projection output (K4).

The packed projection writes ``[tokens, (H + 2*KV) * D]``; the first ``H + KV`` heads (q then k)
are rotated in place, v passes through.  cos/sin tables are precomputed on the host in fp32
(``RotaryTable``) -- the kernel does no trig.  Backward is the inverse rotation of the incoming
gradient, also in place (the qkv activation itself is never saved: attention saves q/k/v).
"""
from __future__ import annotations

import math

import torch

from ._backend import ext, use_hip


class RotaryTable:
    """fp32 cos/sin tables ``[max_pos, head_dim/2]`` (HF rotate_half convention)."""

    def __init__(self, head_dim: int, max_pos: int, theta: float = 10000.0, scaling: dict | None = None):
        self.head_dim, self.max_pos, self.theta = head_dim, max_pos, theta
        inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
        if scaling and scaling.get("rope_type") == "llama3":
            inv = _llama3_scale(inv, scaling)
        t = torch.arange(max_pos, dtype=torch.float64)
        f = torch.outer(t, inv)
        self._cpu = (f.cos().float().contiguous(), f.sin().float().contiguous())
        self._dev: dict[torch.device, tuple[torch.Tensor, torch.Tensor]] = {}

    def get(self, device: torch.device):
        device = torch.device(device)
        if device.type == "cpu":
            return self._cpu
        if device not in self._dev:
            self._dev[device] = tuple(t.to(device) for t in self._cpu)
        return self._dev[device]


def _llama3_scale(inv: torch.Tensor, sc: dict) -> torch.Tensor:
    """Llama-3.1 frequency scaling (applied only when a config asks for it)."""
    factor = sc.get("factor", 8.0)
    lo, hi = sc.get("low_freq_factor", 1.0), sc.get("high_freq_factor", 4.0)
    old = sc.get("original_max_position_embeddings", 8192)
    lo_wl, hi_wl = old / lo, old / hi
    wl = 2 * math.pi / inv
    out = torch.where(wl > lo_wl, inv / factor, inv)
    smooth = (old / wl - lo) / (hi - lo)
    mid = (1 - smooth) * out / factor + smooth * out
    is_mid = (wl >= hi_wl) & (wl <= lo_wl)
    return torch.where(is_mid, mid, out)


def _rope_ref(qkv: torch.Tensor, cos, sin, n_rot: int, D: int, seq_len: int, positions, inverse: bool):
    T = qkv.shape[0]
    pos = positions.long() if positions is not None else torch.arange(T, device=qkv.device) % seq_len
    c = cos.to(qkv.device)[pos].unsqueeze(1)  # [T,1,D/2]
    s = sin.to(qkv.device)[pos].unsqueeze(1)
    if inverse:
        s = -s
    x = qkv[:, : n_rot * D].float().view(T, n_rot, D)
    x1, x2 = x[..., : D // 2], x[..., D // 2 :]
    rot = torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).view(T, n_rot * D)
    out = qkv.clone()
    out[:, : n_rot * D] = rot.to(qkv.dtype)
    return out


class _RopeHip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, n_rot, D, seq_len, positions, handoff=None):
        ext().rope_(qkv, cos, sin, positions, n_rot, D, seq_len, False)
        ctx.mark_dirty(qkv)
        ctx.args = (cos, sin, n_rot, D, seq_len, positions)
        ctx.handoff = handoff
        return qkv

    @staticmethod
    def backward(ctx, g):
        if ctx.handoff is not None and ctx.handoff.taken:  # the flash backward emitted un-rotated dq / dk
            return g, None, None, None, None, None, None, None
        cos, sin, n_rot, D, seq_len, positions = ctx.args
        if g.dim() != 2 or g.stride(1) != 1 or g.stride(0) % 8:
            g = g.contiguous()  # (a row-padded 2-D view is rotated in place, keeping its spare columns)
        ext().rope_(g, cos, sin, positions, n_rot, D, seq_len, True)
        return g, None, None, None, None, None, None, None


def apply_rope_packed(qkv: torch.Tensor, table: RotaryTable, n_q: int, n_kv: int, head_dim: int, seq_len: int,
                      positions: torch.Tensor | None = None, handoff=None) -> torch.Tensor:
    """Rotate q and k heads of a packed ``[T, (H+2KV)*D]`` projection (in place on GPU).  ``handoff``
    (GPU path): an ``ops.attention.RopeGrad`` given to the consuming attention -- when the flash
    backward takes it, this op's backward is the identity (dq / dk arrive un-rotated)."""
    cos, sin = table.get(qkv.device)
    n_rot = n_q + n_kv
    if use_hip(qkv) and qkv.dtype == torch.bfloat16:
        if positions is not None:
            positions = positions.to(torch.int32).contiguous()
        return _RopeHip.apply(qkv, cos, sin, n_rot, head_dim, seq_len, positions, handoff)
    return _rope_ref(qkv, cos, sin, n_rot, head_dim, seq_len, positions, False)
