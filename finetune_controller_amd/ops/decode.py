"""KV cache + decode attention for generation (``models.generate``).

``KVCache`` keeps, per layer, ``[B, Lmax, KV*D]`` bf16 K and V rows (post-RoPE) plus each
sequence's length.  Prefill writes a prompt's rows with the ordinary (flash) causal attention; every
decode step appends one row per sequence and attends with ``decode_attention``:

* GPU: ``csrc/kernels/decode_attn.hip`` -- split-K flash decoding over 256-key chunks, the G query
  heads of a kv group scored against each cached row in one pass, a deterministic combine kernel;
* CPU / ``FTC_KERNELS=torch``: the masked-softmax reference below (also the numerics oracle).
"""
from __future__ import annotations

import math

import torch

from ._backend import ext, use_hip


def decode_attention_reference(q, k_cache, v_cache, lens, H: int, KV: int, D: int, scale: float,
                               window: int = 0) -> torch.Tensor:
    """q [B, >=H*D]; caches [B, Lmax, KV*D]; lens [B] valid keys -> [B, H*D] (fp32 math)."""
    B, L = k_cache.shape[0], k_cache.shape[1]
    G = H // KV
    qf = q[:, :H * D].float().view(B, KV, G, D)
    k = k_cache.float().view(B, L, KV, D)
    v = v_cache.float().view(B, L, KV, D)
    s = torch.einsum("bkgd,blkd->bkgl", qf, k) * scale
    t = torch.arange(L, device=q.device)
    n = lens.to(q.device).long().view(B, 1)
    ok = t[None, :] < n
    if window and window > 0:
        ok &= t[None, :] >= (n - window)
    s = s.masked_fill(~ok[:, None, None, :], float("-inf"))
    p = s.softmax(-1)
    o = torch.einsum("bkgl,blkd->bkgd", p, v)
    return o.reshape(B, H * D).to(q.dtype)


def decode_attention(qkv, k_cache, v_cache, lens, max_len: int, H: int, KV: int, D: int, scale: float | None = None,
                     window: int = 0) -> torch.Tensor:
    """One query token per sequence against its cache.  ``qkv`` [B, (H+2KV)*D]: the current token's
    packed projection, whose K / V rows are appended at position ``lens - 1`` (the HIP kernel does it
    while attending); ``max_len`` (host int) bounds ``lens``."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if use_hip(qkv) and qkv.dtype == torch.bfloat16 and D in (64, 128) and H // KV <= 8:
        return ext().decode_attention(qkv, k_cache, v_cache, lens, H, KV, D, int(max_len), scale, int(window or 0))
    B, kv = qkv.shape[0], KV * D
    rows, pos = torch.arange(B, device=qkv.device), lens.long() - 1
    k_cache.index_put_((rows, pos), qkv[:, H * D:H * D + kv])
    v_cache.index_put_((rows, pos), qkv[:, H * D + kv:H * D + 2 * kv])
    return decode_attention_reference(qkv, k_cache, v_cache, lens, H, KV, D, scale, window)


class KVCache:
    """Per-layer K/V rows of B sequences.  ``lens`` (device int32) and ``host_lens`` (python ints,
    so no step needs a device read) advance together."""

    def __init__(self, n_layers: int, B: int, max_len: int, KV: int, D: int, device, dtype=torch.bfloat16):
        self.k = torch.zeros(n_layers, B, max_len, KV * D, device=device, dtype=dtype)
        self.v = torch.zeros_like(self.k)
        self.B, self.max_len, self.KV, self.D = B, max_len, KV, D
        self.lens = torch.zeros(B, dtype=torch.int32, device=device)
        self.host_lens = [0] * B
        self.row: int | None = None  # prefill of ONE sequence (batch row) at a time
        self.decoding = False
        self.graph_mode = False  # decode steps replayed from a hipGraph: attend over the full capacity

    def store(self, layer: int, qkv: torch.Tensor, H: int, S: int):
        """Prefill: write rows [0, S) of sequence ``self.row`` (decode steps append inside
        ``decode_attention``)."""
        kv = self.KV * self.D
        self.k[layer, self.row, :S].copy_(qkv[:, H * self.D:H * self.D + kv].view(S, kv))
        self.v[layer, self.row, :S].copy_(qkv[:, H * self.D + kv:H * self.D + 2 * kv].view(S, kv))

    def begin_decode(self):
        """Positions of the tokens about to be appended (= current lengths); ``lens_next`` (their
        lengths once appended) is formed once per step for every layer's attention."""
        self.decoding = True
        self.lens_next = self.lens + 1
        return self.lens  # RoPE positions, int32 [B]

    def attend_len(self) -> int:
        """Host bound on the lengths of this decode step: the exact maximum eagerly, the capacity
        under graph replay (the split count is part of the captured launch; chunks past a
        sequence's length exit at once)."""
        return self.max_len if self.graph_mode else max(self.host_lens) + 1

    def end_decode(self):
        self.lens += 1
        self.host_lens = [n + 1 for n in self.host_lens]

    def finish_prefill(self, row: int, n: int):
        self.lens[row] = n
        self.host_lens[row] = n
