"""SwiGLU (K9) for Llama/Mistral MLPs and GELU for GPT-2.

``swiglu(gu)`` consumes the packed gate|up projection ``[T, 2F]`` and returns ``silu(g) * u``.
The backward recomputes silu from the saved ``gu`` (the [T, F] product is never saved).
With LoRA on the neighbouring projections the kernels also form the rank-r tail products of the
augmented GEMMs (``ops.linear``) from the values they produce, saving a full re-read of h / dgu.
"""
from __future__ import annotations


import torch
import torch.nn.functional as F

from ._backend import ext, use_hip
from .linear import LoRATail, gate_wgrad_stream, mark_prefilled

_FUSED_OFF = False  # True: separate tail GEMMs (A/B by patching; profiles/r1_bench_fused_swiglu_tail*.log)


class _SwiGLUHip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu, out_pad, grad_pad, fwd_tail, bwd_tail):
        gu2 = gu.reshape(-1, gu.shape[-1])
        ctx.save_for_backward(gu2)
        ctx.shp, ctx.grad_pad, ctx.bwd_tail = gu.shape, grad_pad, bwd_tail
        if fwd_tail is not None:
            # h and s h A_down^T in one pass (csrc/kernels/swiglu_lora.hip); the down projection's
            # augmented GEMM then finds its tail columns already formed
            t = fwd_tail
            a = ext().swiglu_fwd_lora(gu2, out_pad, t.aug.fwd_tail_operand(t.A, t.B, t.scale), t.aug.nct)
            mark_prefilled("fwd", a, t.aug)
            return a
        a = ext().swiglu_fwd(gu2, out_pad)
        return a if out_pad else a.view(*gu.shape[:-1], gu.shape[-1] // 2)

    @staticmethod
    def backward(ctx, da):
        (gu2,) = ctx.saved_tensors
        da2 = da.reshape(-1, da.shape[-1])
        t = ctx.bwd_tail
        if t is not None and da2.stride(1) == 1 and da2.stride(0) % 8 == 0:
            dgu = ext().swiglu_bwd_lora(da2, gu2, ctx.grad_pad, t.aug.bwd_tail_operand(t.A, t.B, t.scale), t.aug.nct,
                                        t.split)
            mark_prefilled("bwd", dgu, t.aug)
            return dgu, None, None, None, None
        gate_wgrad_stream()
        dgu = ext().swiglu_bwd(da2.contiguous(), gu2, ctx.grad_pad)
        return (dgu if ctx.grad_pad else dgu.view(ctx.shp)), None, None, None, None


def _tail_ok(t: LoRATail | None, pad: int, width: int, rows: int) -> bool:
    # (the kernels make their buffer resources per row block: any number of rows)
    return t is not None and t.aug.Rp == pad and t.aug.R <= 64 and width % 128 == 0 and not _FUSED_OFF


def swiglu(gu: torch.Tensor, out_pad: int = 0, grad_pad: int = 0, fwd_tail: LoRATail | None = None,
           bwd_tail: LoRATail | None = None) -> torch.Tensor:
    """``silu(g) * u``.  ``out_pad`` / ``grad_pad`` (2-D only): the output / the gradient of ``gu``
    are column views of row-padded buffers (spare columns for the augmented LoRA GEMMs).
    ``fwd_tail`` (the down projection's LoRA) / ``bwd_tail`` (the gate|up projection's LoRA): the
    kernel also forms ``s h A^T`` / ``dgu B`` into those spare columns."""
    if use_hip(gu) and gu.dtype == torch.bfloat16 and gu.is_contiguous():
        if gu.dim() != 2:
            out_pad = grad_pad = 0
        F2 = gu.shape[-1]
        rows = gu.numel() // F2
        ft = fwd_tail if _tail_ok(fwd_tail, out_pad, F2 // 2, rows) else None
        bt = bwd_tail if _tail_ok(bwd_tail, grad_pad, F2 // 2, rows) else None
        return _SwiGLUHip.apply(gu, out_pad, grad_pad, ft, bt)
    g, u = gu.chunk(2, dim=-1)
    return F.silu(g) * u


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x, approximate="tanh")
