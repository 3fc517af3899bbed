"""SwiGLU (K9) for Llama/Mistral MLPs and GELU for GPT-2.

``swiglu(gu)`` consumes the packed gate|up projection ``[T, 2F]`` and returns ``silu(g) * u``.
The backward recomputes silu from the saved ``gu`` (the [T, F] product is never saved).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._backend import ext, use_hip


class _SwiGLUHip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, out_pad, grad_pad):
        gu2 = gu.reshape(-1, gu.shape[-1])
        ctx.save_for_backward(gu2)
        ctx.shp, ctx.grad_pad = gu.shape, grad_pad
        a = ext().swiglu_fwd(gu2, out_pad)
        return a if out_pad else a.view(*gu.shape[:-1], gu.shape[-1] // 2)

    @staticmethod
    def backward(ctx, da):
        (gu2,) = ctx.saved_tensors
        dgu = ext().swiglu_bwd(da.reshape(-1, da.shape[-1]).contiguous(), gu2, ctx.grad_pad)
        return (dgu if ctx.grad_pad else dgu.view(ctx.shp)), None, None


def swiglu(gu: torch.Tensor, out_pad: int = 0, grad_pad: int = 0) -> torch.Tensor:
    """``silu(g) * u``.  ``out_pad`` / ``grad_pad`` (2-D only): the output / the gradient of ``gu``
    are column views of row-padded buffers (spare columns for the augmented LoRA GEMMs)."""
    if use_hip(gu) and gu.dtype == torch.bfloat16 and gu.is_contiguous():
        if gu.dim() != 2:
            out_pad = grad_pad = 0
        return _SwiGLUHip.apply(gu, out_pad, grad_pad)
    g, u = gu.chunk(2, dim=-1)
    return F.silu(g) * u


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x, approximate="tanh")
