"""Causal (optionally sliding-window) GQA attention over a packed qkv projection (K1/K2).

``attention_packed(qkv, B, S, H, KV, D)`` takes the ``[B*S, (H+2KV)*D]`` projection output
(q heads, then k heads, then v heads -- the layout the packed Wqkv GEMM writes) and returns the
``[B*S, H*D]`` attention output that feeds the o-projection GEMM directly.  q/k/v are consumed as
strided views: nothing is transposed or copied.

GPU: the gfx950 flash-attention kernels (``csrc/kernels/flash_attn.hip``: MFMA bf16, LDS-tiled K/V,
online softmax, LSE saved for the backward, GQA handled by mapping q heads onto their kv head).
The backward writes dq/dk/dv straight into ONE packed ``dqkv`` buffer, which is the gradient of the
packed projection output -- again no concatenation.

CPU / ``FTC_KERNELS=torch``: ``torch.nn.functional.scaled_dot_product_attention``.

Packed sequences (several documents per row, ``Segments``): a query sees only keys of its own
document.  The kernels take per-token document bounds -- ``doc_start`` for the query-on-lane passes
(forward, dQ), ``doc_end`` for the key-on-lane dK/dV pass -- skip key / query tiles outside the
document range and mask per element only on tiles that straddle a boundary.
"""
from __future__ import annotations

import logging
import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from ._backend import ext, use_hip
from .linear import gate_wgrad_stream as _gate_dw


# flipped to True once csrc/kernels/flash_attn.hip replaces the stub launcher
FLASH_READY = True
FLASH_TILE = 256  # the kernels' query/key tile: S must be a multiple natively
_log = logging.getLogger("ftc.attention")
_WARNED: set = set()


def flash_supported(D: int, S: int) -> bool:
    """The kernels run this shape natively (no tail padding)."""
    return FLASH_READY and D in (64, 128) and S % FLASH_TILE == 0


def flash_usable(D: int, S: int, causal: bool) -> bool:
    """The flash path handles this shape: natively, or through padding (``_FlashPaddedTail``): S not a
    multiple of the tile gets tail rows (causal attention never sees the pads; non-causal attention
    masks keys past S in the kernels, ``kv_valid``), a head_dim the kernels are not built for (80, 96,
    112, ... any D <= 128) gets zero columns up to the next kernel head_dim."""
    return FLASH_READY and 0 < D <= 128


def kernel_head_dim(D: int) -> int:
    """The kernels' head_dim a D <= 128 head runs at (zero-padded columns: exact, see _FlashPaddedTail)."""
    return 64 if D <= 64 else 128


def model_tile_len(S: int, D: int, hip: bool, dtype: torch.dtype, max_len: int) -> int:
    """Sequence length a whole causal LM should run at on the GPU: S rounded up to the flash tile
    when S is not a multiple of it (and the rounded length stays within the position range).

    Padding at the MODEL input instead of inside attention keeps every kernel on its tile-aligned
    fast path (T = B*Sp rows for hipBLASLt, the split-T LoRA weight-gradient kernels, native flash):
    measured at 4 x 4000 tokens, attention-only tail padding ran the step 12 % slower than 4 x 4096
    (profiles/r2/prof_tail4000_attention_only.md), model-level padding costs the padded tokens'
    compute only.  Exact for causal models: pads sit at the END of each row, so no real position
    attends to them, and their labels are ignored."""
    if not hip or dtype != torch.bfloat16 or not 0 < D <= 128 or S % FLASH_TILE == 0:
        return S
    Sp = -(-S // FLASH_TILE) * FLASH_TILE
    return Sp if Sp <= max_len else S


def pad_batch_to(Sp: int, input_ids: torch.Tensor, labels: torch.Tensor | None = None, positions=None,
                 segments: "Segments | None" = None, pad_id: int = 0):
    """Right-pad a [B, S] batch to Sp positions: pad tokens ``pad_id``, labels -100 (ignored by the
    loss), positions continue, and the pads form one extra document per row when packed."""
    B, S = input_ids.shape
    ids = F.pad(input_ids, (0, Sp - S), value=pad_id)
    if labels is not None:
        labels = F.pad(labels.reshape(B, S), (0, Sp - S), value=-100)
    if positions is not None:
        pos = positions.reshape(-1, S)
        tail = torch.arange(S, Sp, device=pos.device, dtype=pos.dtype).expand(pos.shape[0], Sp - S)
        positions = torch.cat([pos, tail], 1).reshape(-1) if positions.dim() == 1 else torch.cat([pos, tail], 1)
    if segments is not None:
        segments = _pad_segments(segments, B, S, Sp)
    return ids, labels, positions, segments


def _warn_fallback(reason: str):
    if reason not in _WARNED:
        _WARNED.add(reason)
        _log.warning("attention: falling back to torch SDPA on the GPU (%s) -- about 3x slower than the "
                     "gfx950 flash kernels", reason)


@dataclass
class Segments:
    """Document layout of a packed [B, S] batch, int32 flat [B*S] (positions within the row):
    ``doc_start[t]`` first position of t's document, ``doc_end[t]`` one past its last, ``positions[t]``
    = t - doc_start[t] (RoPE / learned positions restart per document)."""

    doc_start: torch.Tensor
    doc_end: torch.Tensor
    positions: torch.Tensor


def segments_from_eos(ids: torch.Tensor, eos_id: int) -> Segments:
    """Documents end at (and include) each ``eos_id`` token; computed on the ids' device (cummax /
    cummin scans, no host sync)."""
    B, S = ids.shape
    t = torch.arange(S, device=ids.device, dtype=torch.int64).expand(B, S)
    is_eos = ids == eos_id
    starts = torch.zeros_like(is_eos)
    starts[:, 0] = True
    starts[:, 1:] = is_eos[:, :-1]
    doc_start = torch.where(starts, t, torch.zeros_like(t)).cummax(dim=1).values
    ends = is_eos.clone()
    ends[:, -1] = True
    last = torch.where(ends, t, torch.full_like(t, S)).flip(1).cummin(dim=1).values.flip(1)
    doc_end = last + 1
    return Segments(doc_start.to(torch.int32).reshape(-1).contiguous(), doc_end.to(torch.int32).reshape(-1).contiguous(),
                    (t - doc_start).to(torch.int32).reshape(-1).contiguous())


def _doc_mask(docs: Segments, B: int, S: int) -> torch.Tensor:
    """[B, 1, S, S] bool: causal and same document."""
    ds = docs.doc_start.view(B, S).long()
    k = torch.arange(S, device=ds.device)
    return ((k[None, None, :] <= k[None, :, None]) & (k[None, None, :] >= ds[:, :, None])).unsqueeze(1)


def _split(qkv, B, S, H, KV, D):
    q = qkv[:, : H * D]
    k = qkv[:, H * D : (H + KV) * D]
    v = qkv[:, (H + KV) * D : (H + 2 * KV) * D]
    return q, k, v


def _sdpa_packed(qkv, B, S, H, KV, D, causal, window, scale, docs: Segments | None = None):
    q, k, v = _split(qkv, B, S, H, KV, D)
    q = q.reshape(B, S, H, D).transpose(1, 2)
    k = k.reshape(B, S, KV, D).transpose(1, 2)
    v = v.reshape(B, S, KV, D).transpose(1, 2)
    if KV != H:
        rep = H // KV
        k = k.repeat_interleave(rep, dim=1)
        v = v.repeat_interleave(rep, dim=1)
    mask = None
    if docs is not None:
        mask = _doc_mask(docs, B, S)
        if window and window > 0:
            i = torch.arange(S, device=qkv.device)
            mask = mask & ((i[:, None] - i[None, :]) < window)
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, scale=scale)
    elif window and window > 0 and window < S:
        i = torch.arange(S, device=qkv.device)
        allowed = (i[None, :] <= i[:, None]) & (i[:, None] - i[None, :] < window)
        mask = allowed
        o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, scale=scale)
    else:
        o = F.scaled_dot_product_attention(q, k, v, is_causal=causal, scale=scale)
    return o.transpose(1, 2).reshape(B * S, H * D)


# RoPE-backward handoff to the flash epilogues (False: the producer runs the separate pass; tests patch it)
ROPE_BWD_FUSE = True


class RopeGrad:
    """Handoff between a producer that applied RoPE to the packed q / k heads (``ops.lora_linear(...,
    rope=)``) and this attention: when the flash path runs it takes the rotation's backward into the dQ /
    dK epilogues (``taken``; csrc/kernels/flash_attn_bwd.hip ``rope_inv_rows``) and the producer's
    backward skips its separate inverse-rotation pass over dq / dk.  Positions: ``pos`` int32 [B*S] or
    the row index within its sequence."""

    __slots__ = ("cos", "sin", "pos", "taken")

    def __init__(self, cos: torch.Tensor, sin: torch.Tensor, pos: torch.Tensor | None):
        self.cos, self.sin, self.pos, self.taken = cos, sin, pos, False


class _FlashPacked(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B, S, H, KV, D, causal, window, scale, out_pad=0, grad_pad=0, docs=None, rope_grad=None):
        q, k, v = _split(qkv, B, S, H, KV, D)
        o, lse = ext().flash_fwd(q, k, v, B, S, H, KV, D, scale, causal, window, out_pad,
                                 docs.doc_start if docs is not None else None)
        # o is kept outside save_for_backward: with out_pad the consumer writes its LoRA activations
        # into the spare columns of o's buffer, which bumps the shared version counter (the [:, :H*D]
        # values themselves never change)
        ctx.save_for_backward(qkv, lse)
        ctx.o = o.detach()
        ctx.cfg = (B, S, H, KV, D, causal, window, scale)
        ctx.grad_pad = grad_pad
        ctx.docs = docs
        ctx.rope_grad = None
        if rope_grad is not None and ROPE_BWD_FUSE and D == 128 and rope_grad.cos.shape[-1] == 64 and (
                rope_grad.pos is not None or rope_grad.cos.shape[0] >= S):
            rope_grad.taken = True
            ctx.rope_grad = rope_grad
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, lse = ctx.saved_tensors
        o = ctx.o
        B, S, H, KV, D, causal, window, scale = ctx.cfg
        if do.stride(-1) != 1 or do.stride(0) % 8:
            do = do.contiguous()
        q, k, v = _split(qkv, B, S, H, KV, D)
        Wd = qkv.shape[1]
        # grad_pad: dqkv is a column view of a row-padded buffer (spare columns for the augmented
        # LoRA backward GEMM of the qkv projection)
        dqkv = torch.empty(qkv.shape[0], Wd + ctx.grad_pad, dtype=qkv.dtype, device=qkv.device)[:, :Wd]
        dq, dk, dv = _split(dqkv, B, S, H, KV, D)
        docs = ctx.docs
        rg = ctx.rope_grad
        _gate_dw()
        ext().flash_bwd(q, k, v, o, do, lse, dq, dk, dv, B, S, H, KV, D, scale, causal, window,
                        docs.doc_start if docs is not None else None, docs.doc_end if docs is not None else None,
                        -1, rg.cos if rg is not None else None, rg.sin if rg is not None else None,
                        rg.pos if rg is not None else None)
        return dqkv, None, None, None, None, None, None, None, None, None, None, None, None


def _pad_segments(docs: Segments, B: int, S: int, Sp: int) -> Segments:
    """Document bounds of the tail-padded rows: the pad positions form one extra document per row."""
    def pad(t, fill):
        out = torch.full((B, Sp), fill, dtype=t.dtype, device=t.device)
        out[:, :S] = t.view(B, S)
        return out.reshape(-1)
    ds = pad(docs.doc_start, S)
    de = pad(docs.doc_end, Sp)
    return Segments(ds, de, pad(docs.positions, 0))


def _pad_heads(t: torch.Tensor, B: int, S: int, Sp: int, nh: int, D: int, Dp: int) -> torch.Tensor:
    """[B*S, nh*D] (any row stride) -> zero-padded [B*Sp, nh*Dp]: rows S..Sp and head columns D..Dp zero."""
    out = t.new_zeros(B, Sp, nh, Dp)
    out[:, :S, :, :D].copy_(t.reshape(B, S, nh, D) if t.is_contiguous() else t.unflatten(0, (B, S)).unflatten(2, (nh, D)))
    return out.view(B * Sp, nh * Dp)


def _unpad_heads(t: torch.Tensor, out: torch.Tensor, B: int, S: int, Sp: int, nh: int, D: int, Dp: int):
    """Inverse of _pad_heads into the (column-view) ``out`` [B*S, nh*D]."""
    out.unflatten(0, (B, S)).unflatten(2, (nh, D)).copy_(t.view(B, Sp, nh, Dp)[:, :S, :, :D])


class _FlashPaddedTail(torch.autograd.Function):
    """Flash attention on a padded copy of the problem, for shapes the kernels do not take natively.

    * S not a multiple of the 256-row tile: each row is padded to Sp = ceil(S/256)*256 with zero q/k/v
      rows at the END.  Exact: under the causal mask no real query (position < S) sees a pad key
      (position >= S); without it the kernels mask every key >= S (``kv_valid``: forward and dQ pass).
      Pad queries' outputs are dropped and their output gradient is zero, so they add nothing to dK/dV;
      the pads of a packed-document batch form a document of their own.
    * head_dim D not in {64, 128} (D <= 128): every head is zero-padded to Dp = kernel_head_dim(D)
      columns, with the softmax scale of the real D.  Exact: zero q/k columns add nothing to QK^T, zero
      v columns give zero output columns (dropped), the zero output-gradient columns add nothing to dP
      or delta, and the dq/dk/dv pad columns are dropped.
    Costs one copy of qkv / o / do / dqkv per call (about a tenth of the attention time at S ~ 4k; the
    head pad adds (Dp - D) / D of the attention FLOPs) instead of the 3x slower SDPA fallback."""

    @staticmethod
    def forward(ctx, qkv, B, S, H, KV, D, window, scale, out_pad=0, grad_pad=0, docs=None, causal=True):
        Sp = -(-S // FLASH_TILE) * FLASH_TILE
        Dp = kernel_head_dim(D)
        nh = H + 2 * KV
        if Dp == D:
            W = qkv.shape[1]
            qkv_p = qkv.new_zeros(B, Sp, W)
            qkv_p[:, :S].copy_(qkv.unflatten(0, (B, S)))
            qkv_p = qkv_p.view(B * Sp, W)
        else:
            qkv_p = _pad_heads(qkv, B, S, Sp, nh, D, Dp)
        docs_p = _pad_segments(docs, B, S, Sp) if docs is not None and Sp != S else docs
        q, k, v = _split(qkv_p, B, Sp, H, KV, Dp)
        # causal: the pads are invisible to every real query as they are (and masking them would leave
        # late pad queries under a window with no key at all); non-causal: mask keys >= S in the kernels
        kv_valid = -1 if causal or Sp == S else S
        o_p, lse = ext().flash_fwd(q, k, v, B, Sp, H, KV, Dp, scale, causal, window, 0,
                                   docs_p.doc_start if docs_p is not None else None, kv_valid)
        HD = H * D
        out = torch.empty(B * S, HD + out_pad, dtype=qkv.dtype, device=qkv.device)[:, :HD]
        if Dp == D:
            out.unflatten(0, (B, S)).copy_(o_p.view(B, Sp, HD)[:, :S])
        else:
            _unpad_heads(o_p, out, B, S, Sp, H, D, Dp)
        ctx.save_for_backward(qkv_p, o_p, lse)
        ctx.cfg = (B, S, Sp, H, KV, D, Dp, window, scale, grad_pad, causal, qkv.shape[1])
        ctx.docs = docs_p
        return out

    @staticmethod
    def backward(ctx, do):
        qkv_p, o_p, lse = ctx.saved_tensors
        B, S, Sp, H, KV, D, Dp, window, scale, grad_pad, causal, W = ctx.cfg
        HD = H * D
        if Dp == D:
            do_p = do.new_zeros(B, Sp, HD)
            do_p[:, :S].copy_(do.unflatten(0, (B, S)))
            do_p = do_p.view(B * Sp, HD)
        else:
            do_p = _pad_heads(do, B, S, Sp, H, D, Dp)
        dqkv_p = torch.empty_like(qkv_p)
        q, k, v = _split(qkv_p, B, Sp, H, KV, Dp)
        dq, dk, dv = _split(dqkv_p, B, Sp, H, KV, Dp)
        docs = ctx.docs
        _gate_dw()
        ext().flash_bwd(q, k, v, o_p, do_p, lse, dq, dk, dv, B, Sp, H, KV, Dp, scale, causal, window,
                        docs.doc_start if docs is not None else None, docs.doc_end if docs is not None else None,
                        -1 if causal or Sp == S else S)
        dqkv = torch.empty(B * S, W + grad_pad, dtype=qkv_p.dtype, device=qkv_p.device)[:, :W]
        if Dp == D:
            dqkv.unflatten(0, (B, S)).copy_(dqkv_p.view(B, Sp, W)[:, :S])
        else:
            _unpad_heads(dqkv_p, dqkv, B, S, Sp, H + 2 * KV, D, Dp)
        return dqkv, None, None, None, None, None, None, None, None, None, None, None


def attention_packed(qkv: torch.Tensor, B: int, S: int, H: int, KV: int, D: int, causal: bool = True,
                     window: int = 0, scale: float | None = None, out_pad: int = 0,
                     grad_pad: int = 0, docs: Segments | None = None,
                     rope_grad: RopeGrad | None = None) -> torch.Tensor:
    """Causal / sliding-window GQA attention on a packed ``[B*S, (H+2KV)*D]`` projection.

    ``out_pad`` / ``grad_pad``: the output / the gradient of ``qkv`` are column views of
    row-padded buffers (spare columns for the augmented LoRA GEMMs, ``ops.linear``).  ``docs``: packed
    documents (causal only).  ``rope_grad``: see :class:`RopeGrad` (taken on the untiled flash path)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if docs is not None and not causal:
        raise ValueError("document-masked attention is causal")
    if use_hip(qkv):
        if qkv.dtype == torch.bfloat16 and flash_supported(D, S):
            return _FlashPacked.apply(qkv, B, S, H, KV, D, causal, int(window or 0), scale, out_pad, grad_pad, docs,
                                      rope_grad)
        if qkv.dtype == torch.bfloat16 and flash_usable(D, S, causal):
            return _FlashPaddedTail.apply(qkv, B, S, H, KV, D, int(window or 0), scale, out_pad, grad_pad, docs,
                                          bool(causal))
        _warn_fallback(f"dtype={qkv.dtype}, head_dim={D}, seq_len={S}, causal={causal}")
    return _sdpa_packed(qkv, B, S, H, KV, D, causal, window, scale, docs)


def attention_reference(qkv, B, S, H, KV, D, causal=True, window=0, scale=None, docs: Segments | None = None):
    """fp32 math reference used by the kernel numerics tests."""
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    q, k, v = (t.float() for t in _split(qkv, B, S, H, KV, D))
    q = q.reshape(B, S, H, D).transpose(1, 2)
    k = k.reshape(B, S, KV, D).transpose(1, 2).repeat_interleave(H // KV, dim=1)
    v = v.reshape(B, S, KV, D).transpose(1, 2).repeat_interleave(H // KV, dim=1)
    s = (q @ k.transpose(-1, -2)) * scale
    i = torch.arange(S, device=qkv.device)
    allowed = torch.ones(S, S, dtype=torch.bool, device=qkv.device)
    if causal:
        allowed &= i[None, :] <= i[:, None]
    if window and window > 0:
        allowed &= (i[:, None] - i[None, :]) < window
    if docs is not None:
        allowed = allowed & _doc_mask(docs, B, S)
    s = s.masked_fill(~allowed, float("-inf"))
    p = s.softmax(-1)
    return (p @ v).transpose(1, 2).reshape(B * S, H * D)
