"""RMSNorm with the residual add fused in (K3), plus LayerNorm for GPT-2 (K11).

``add_rms_norm(h, delta, w)`` returns ``(h + delta, rmsnorm(h + delta) * w)`` -- the decoder
layers keep the residual stream ``h`` and every norm consumes the preceding sub-block output
``delta`` in the same pass, so the residual add never costs its own HBM round trip.
On GPU both directions run the gfx950 kernels of ``csrc/kernels/rmsnorm.hip``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._backend import ext, use_hip
from .linear import gate_wgrad_stream


def _rms_ref(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    r = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * r * w.float()).to(x.dtype)


class _AddRMSNormHip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, delta, w, eps, pad, grad_pad):
        shp = h.shape
        h2 = h.reshape(-1, shp[-1])
        d2 = delta.reshape(-1, shp[-1]) if delta is not None else None
        y, rstd, hn = ext().rmsnorm_fwd(h2, d2, w, eps, pad)
        ctx.save_for_backward(hn, w, rstd)
        ctx.has_delta = delta is not None
        ctx.shp = shp
        ctx.grad_pad = grad_pad if (delta is not None and h.dim() == 2) else 0
        return hn.view(shp), (y if pad else y.view(shp))

    @staticmethod
    def backward(ctx, dh_out, dy):
        hn, w, rstd = ctx.saved_tensors
        d = ctx.shp[-1]
        dy2 = dy.reshape(-1, d).contiguous()
        dres = None
        if dh_out is not None:
            dres = dh_out.reshape(-1, d)
            if dres.stride(1) != 1 or dres.stride(0) % 8 or dres.data_ptr() % 16:
                dres = dres.contiguous()  # (row-padded views from the next norm are read in place)
        need_dw = ctx.needs_input_grad[2]
        gate_wgrad_stream()
        outs = ext().rmsnorm_bwd(dy2, hn, w, rstd, dres, need_dw, ctx.grad_pad)
        dx = outs[0] if ctx.grad_pad else outs[0].view(ctx.shp)
        dw = outs[1].to(w.dtype) if need_dw else None
        return dx, (dx if ctx.has_delta else None), dw, None, None, None


def add_rms_norm(h: torch.Tensor, delta: torch.Tensor | None, w: torch.Tensor, eps: float = 1e-5, pad: int = 0,
                 grad_pad: int = 0):
    """Returns ``(h_new, y)`` with ``h_new = h + delta`` (or ``h``) and ``y = rmsnorm(h_new) * w``.

    ``pad > 0`` (2-D ``h`` only): ``y`` is a column view of a ``[T, d + pad]`` buffer whose spare
    columns the next LoRA projection uses (``ops.linear`` augmented GEMM).  ``grad_pad``: the
    gradient of ``h``/``delta`` is likewise padded, for the augmented backward of the projection
    that produced ``delta``."""
    if use_hip(h) and h.dtype == torch.bfloat16 and w.dtype == torch.bfloat16:
        return _AddRMSNormHip.apply(h, delta, w, eps, pad if h.dim() == 2 else 0, grad_pad)
    hn = h + delta if delta is not None else h
    return hn, _rms_ref(hn, w, eps)


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float = 1e-5) -> torch.Tensor:
    return add_rms_norm(x, None, w, eps)[1]


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, eps: float = 1e-5) -> torch.Tensor:
    """GPT-2 LayerNorm (correctness-only path per SURVEY.md K11: perf irrelevant)."""
    return F.layer_norm(x, (x.shape[-1],), w, b, eps)
