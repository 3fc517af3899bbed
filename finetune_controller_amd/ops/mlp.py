"""Whole Llama MLP block with LoRA on gate|up and down as ONE autograd function (MI355X path).

``y = down(swiglu(gu(x)))`` with both projections augmented (``ops.linear.AugWeight``) and every
adapter weight homed in the flat gradient buffer (``main_grad``).  Owning the block end to end lets the
backward hand each big tensor to exactly one streaming kernel:

forward
  1. ``s x A_gu^T`` into x's spare columns (skinny GEMM), ``gu = [x | s x A_gu^T] [W_gu | B_gu]^T``
  2. ``h = silu(g) u`` and ``s h A_down^T`` in one pass (``swiglu_fwd_lora``)
  3. ``y = [h | s h A_down^T] [W_down | B_down]^T``
backward
  4. ``dy B_down`` into dy's spare columns, ``dh = [dy | dy B_down] [W_down ; s A_down]`` (TN layout)
  5. ``dB_down += dy^T (s h A_down^T)``  (split-T MFMA stream over dy, csrc/kernels/lora_wgrad.hip)
  6. ``swiglu_bwd_wgrad``: dgu, its tail ``dgu B_gu``, ``dB_gu += dgu^T (s x A_gu^T)`` and
     ``dA_down += s (dy B_down)^T h`` -- h recomputed from g, u in registers, so neither dgu (940 MB at
     Llama-3-8B / 16k tokens) nor h (470 MB) is re-read for a weight gradient
  7. ``dx = [dgu | dgu B_gu] [W_gu ; s A_gu]``, ``dA_gu += s x^T (dgu B_gu)``

The unfused composition (``ops.linear.lora_linear`` + ``ops.activation.swiglu``) stays the reference
and the path for every other configuration (QLoRA, LoRA dropout, ranks other than 16 per segment,
optimizers without flat gradient buffers).
"""
from __future__ import annotations

import os

import torch

from ._backend import ext, use_hip
from .linear import _accum_xty, _grad_ready, _spare_cols, _tail, _wide, tail_product, tn_backward

_OFF = os.environ.get("FTC_FUSED_MLP", "1") == "0"  # A/B switch: unfused composition


def fused_mlp_supported(x2: torch.Tensor, aug_gu, pair_gu, aug_down, pair_down, p_gu: int, p_down: int,
                        training: bool) -> bool:
    """True when ``lora_mlp`` can run the fused path for this [T, d] input (padded row view)."""
    if _OFF or not use_hip(x2) or x2.dtype != torch.bfloat16 or x2.dim() != 2:
        return False
    if aug_gu is None or aug_down is None or pair_gu is None or pair_down is None:
        return False
    if training and (pair_gu.dropout > 0.0 or pair_down.dropout > 0.0):
        return False
    F = aug_down.K
    if not (aug_gu.N == 2 * F and aug_down.N == aug_gu.K and p_gu == aug_gu.Rp and p_down == aug_down.Rp):
        return False
    if not (aug_gu.R == 32 and aug_down.R == 16 and aug_gu.Rp >= 32 and aug_down.Rp >= 16):
        return False
    blocks = pair_gu.blocks
    if not (blocks is not None and len(blocks) == 2 and tuple(blocks[0]) == (0, F, 0, 16)
            and tuple(blocks[1]) == (F, 2 * F, 16, 32)):
        return False
    for p in (pair_gu.A, pair_gu.B, pair_down.A, pair_down.B):
        if getattr(p, "main_grad", None) is None:
            return False
    if not _spare_cols(x2, aug_gu.K, aug_gu.Rp):
        return False
    # swiglu_bwd_wgrad's limits (csrc/kernels/swiglu_lora.hip): 512-column blocks, 32-bit buffer offsets
    T, Rp = x2.shape[0], aug_gu.Rp
    return F % 512 == 0 and T * 4 * F < 2 ** 31 and T * (2 * F + Rp) * 2 < 2 ** 31 and Rp % 8 == 0


class _LoRAMLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, A_gu, B_gu, A_dn, B_dn, aug_gu, aug_dn, s_gu, s_dn):
        x2 = x.reshape(-1, x.shape[-1])
        T = x2.shape[0]
        K, N = aug_gu.K, aug_gu.N  # d, 2F
        F, d = aug_dn.K, aug_dn.N
        # 1. gate|up projection, LoRA folded in through x's spare columns
        aug_gu.refresh(A_gu, B_gu, s_gu)
        tail_product(x2, K, aug_gu.Rp, aug_gu.big[N:, :K], aug_gu.nct)
        gu = torch.mm(_wide(x2, K + aug_gu.Rp), aug_gu.big[:N].t())
        # 2. SwiGLU + s h A_down^T into h's spare columns
        h = ext().swiglu_fwd_lora(gu, aug_dn.Rp, aug_dn.fwd_tail_operand(A_dn, B_dn, s_dn), aug_dn.nct)
        # 3. down projection
        y = torch.empty(*x.shape[:-1], d, dtype=x.dtype, device=x.device)
        torch.mm(_wide(h, F + aug_dn.Rp), aug_dn.big[:d].t(), out=y.view(T, d))
        ctx.save_for_backward(x2, gu, h)
        ctx.params = (A_gu, B_gu, A_dn, B_dn)
        ctx.aug, ctx.scales, ctx.shp = (aug_gu, aug_dn), (s_gu, s_dn), x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        x2, gu, h = ctx.saved_tensors
        A_gu, B_gu, A_dn, B_dn = ctx.params
        aug_gu, aug_dn = ctx.aug
        s_gu, s_dn = ctx.scales
        K, N = aug_gu.K, aug_gu.N
        F, d = aug_dn.K, aug_dn.N
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not _spare_cols(dy2, d, aug_dn.Rp):  # the producer gave no spare columns: pad here
            buf = torch.empty(dy2.shape[0], d + aug_dn.Rp, dtype=dy2.dtype, device=dy2.device)
            buf[:, :d].copy_(dy2)
            dy2 = buf[:, :d]
        # 4. dy B_down into dy's spare columns, dh through the augmented TN operand
        aug_dn.refresh(A_dn, B_dn, s_dn)
        tail_product(dy2, d, aug_dn.Rp, aug_dn.bwd_tail_operand(A_dn, B_dn, s_dn), aug_dn.nct)
        dyb_dn = _tail(dy2, d, aug_dn.R)
        rhs = aug_dn.bwd_operand() if tn_backward() else aug_dn.big[:, :F]
        dh = torch.mm(_wide(dy2, d + aug_dn.Rp), rhs)
        # 5. dB_down += dy^T (s h A_down^T)
        _accum_xty(B_dn.main_grad, dy2, _tail(h, F, aug_dn.R), 1.0)
        _grad_ready(B_dn)
        # 6. SwiGLU backward + dgu B_gu + dB_gu + dA_down
        aug_gu.refresh(A_gu, B_gu, s_gu)
        dgu = ext().swiglu_bwd_wgrad(dh, gu, aug_gu.Rp, aug_gu.bwd_tail_operand(A_gu, B_gu, s_gu),
                                     _tail(x2, K, 32), dyb_dn, B_gu.main_grad, A_dn.main_grad, 1.0, s_dn)
        _grad_ready(B_gu)
        _grad_ready(A_dn)
        # 7. dx and dA_gu += s x^T (dgu B_gu)
        dx = None
        if ctx.needs_input_grad[0]:
            rhs = aug_gu.bwd_operand() if tn_backward() else aug_gu.big[:, :K]
            dx = torch.mm(_wide(dgu, N + aug_gu.Rp), rhs).view(ctx.shp)
        _accum_xty(A_gu.main_grad.t(), x2, _tail(dgu, N, aug_gu.R), s_gu)
        _grad_ready(A_gu)
        return dx, None, None, None, None, None, None, None, None


def lora_mlp(x: torch.Tensor, aug_gu, pair_gu, aug_down, pair_down) -> torch.Tensor:
    """Fused LoRA MLP (see module doc).  ``x``: the [T, d] column view of the post-norm buffer with
    ``aug_gu.Rp`` spare columns; call only when ``fused_mlp_supported`` holds."""
    return _LoRAMLPFn.apply(x, pair_gu.A, pair_gu.B, pair_down.A, pair_down.B, aug_gu, aug_down,
                            float(pair_gu.scale), float(pair_down.scale))
