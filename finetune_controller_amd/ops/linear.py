"""Linear layers with LoRA adapters (K5) over packed projections.

``lora_linear(x, W, A, B, scale)`` computes ``y = x W^T + scale * (x A^T) B^T`` with a custom
autograd function that

* never materialises ``W + scale * B A`` (the merged weight) -- the base GEMM runs on the frozen
  weight through hipBLASLt and the rank-r path is two skinny GEMMs;
* saves only ``x`` and the rank-r activation ``xa = x A^T`` for backward;
* skips ``dW`` for a frozen base (LoRA/QLoRA) and, for full fine-tuning, accumulates ``dW``
  directly into the flat gradient buffer (``W.main_grad``) with a beta=1 GEMM instead of
  returning a fresh [out, in] tensor for autograd to add (saves a full read+write of dW).

Packed projections (Wqkv = [q;k;v], Wgu = [gate;up]) carry one LoRA pair per segment.  The
segment A's are stacked (``A = [A_q; A_k; A_v]``, one GEMM for all of them) and the segment B's form
a block-diagonal ``B`` so the LoRA update of the whole packed output is a single GEMM with
K = segments * r.  Off-diagonal blocks of B are structural zeros: their gradient is dropped in the
backward (``lora_blocks``), so they stay exactly zero under AdamW.
"""
from __future__ import annotations

import torch

_GRAD_READY_HOOK = None  # set by parallel.ddp to learn when a main_grad was written


def set_grad_ready_hook(fn):
    global _GRAD_READY_HOOK
    _GRAD_READY_HOOK = fn


def _mask_blocks(dB: torch.Tensor, blocks):
    """Zero everything outside the diagonal blocks [(row0,row1,col0,col1), ...]."""
    if blocks is None:
        return dB
    out = torch.zeros_like(dB)
    for r0, r1, c0, c1 in blocks:
        out[r0:r1, c0:c1] = dB[r0:r1, c0:c1]
    return out


class _LoRALinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, bias, A, B, scale, blocks):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        # allocate the output in its final shape: the returned tensor must not be a view (RoPE
        # rotates it in place downstream)
        out = torch.empty(*shp[:-1], W.shape[0], dtype=x.dtype, device=x.device)
        y = out.view(-1, W.shape[0])
        if bias is None:
            torch.mm(x2, W.t(), out=y)
        else:
            torch.addmm(bias, x2, W.t(), out=y)
        xa = None
        if A is not None:
            xa = x2 @ A.t()
            y.addmm_(xa, B.t(), alpha=scale)
        ctx.save_for_backward(x2, W, A, B, xa)
        ctx.scale, ctx.blocks, ctx.shp, ctx.has_bias = scale, blocks, shp, bias is not None
        return out

    @staticmethod
    def backward(ctx, dy):
        x2, W, A, B, xa = ctx.saved_tensors
        s = ctx.scale
        dy2 = dy.reshape(-1, dy.shape[-1])
        need_x, need_w, need_b, need_a, need_bb = ctx.needs_input_grad[:5]
        dx = dW = db = dA = dB = None
        dyb = None
        if A is not None and (need_x or need_a):
            dyb = dy2 @ B  # [T, R]
        if need_x:
            dx = dy2 @ W
            if dyb is not None:
                dx.addmm_(dyb, A, alpha=s)
            dx = dx.view(ctx.shp)
        if need_w:
            mg = getattr(W, "main_grad", None)
            if mg is not None:
                mg.addmm_(dy2.t(), x2)
                if _GRAD_READY_HOOK is not None:
                    _GRAD_READY_HOOK(W)
            else:
                dW = dy2.t() @ x2
        if need_b and ctx.has_bias:
            db = dy2.sum(0)
        if A is not None:
            if need_bb:
                dB = _mask_blocks(torch.mm(dy2.t(), xa) * s, ctx.blocks)
            if need_a:
                dA = torch.mm(dyb.t(), x2) * s
        return dx, dW, db, dA, dB, None, None


def lora_linear(x: torch.Tensor, W: torch.Tensor, A: torch.Tensor | None = None, B: torch.Tensor | None = None,
                scale: float = 1.0, bias: torch.Tensor | None = None, blocks=None) -> torch.Tensor:
    return _LoRALinearFn.apply(x, W, bias, A, B, scale, blocks)
