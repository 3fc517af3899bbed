"""Chunked fused linear + cross-entropy (K10).

``fused_linear_cross_entropy(h, W, labels)`` = mean over non-ignored rows of
``CE(h @ W^T, labels)`` without ever materialising the ``[tokens, vocab]`` fp32 logits
(Llama-3's vocab 128256 at 16k tokens would be 8.4 GB).  The forward walks the rows in chunks:

  1. ``logits_c = h_c @ W^T``            -- hipBLASLt GEMM into a reusable bf16 chunk buffer
  2. ``ce_fwd_bwd_`` (HIP, in place)      -- per-row loss and ``(softmax - onehot) / n_valid``
  3. ``dh_c = dlogits_c @ W``             -- the input gradient, computed right away
  4. ``W.main_grad += dlogits_c^T @ h_c`` -- only when the lm_head trains (full FT)

so the backward only has to scale the stored ``dh`` by the incoming scalar gradient.  The chunk
buffer is the only vocab-sized allocation.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._backend import ext, use_hip


def _ce_chunk_ref(logits: torch.Tensor, labels: torch.Tensor, gscale: float, ignore_index: int):
    """torch path: returns (loss_rows fp32, dlogits) for one chunk."""
    lf = logits.float()
    lse = torch.logsumexp(lf, dim=-1)
    valid = labels != ignore_index
    safe = torch.where(valid, labels, torch.zeros_like(labels))
    picked = lf.gather(1, safe[:, None]).squeeze(1)
    loss = torch.where(valid, lse - picked, torch.zeros_like(lse))
    p = torch.softmax(lf, dim=-1)
    p.scatter_add_(1, safe[:, None], -valid[:, None].to(p.dtype))
    p *= (valid.to(p.dtype) * gscale)[:, None]
    return loss, p.to(logits.dtype)


class _FusedLinearCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, W, labels, chunk_rows, ignore_index, n_valid_override, grad_enabled=True):
        d = h.shape[-1]
        h2 = h.reshape(-1, d)
        lab = labels.reshape(-1)
        T = h2.shape[0]
        # the normaliser may be fractional: a sequence-parallel shard divides by the whole batch's count / P
        n_valid = float(n_valid_override) if n_valid_override else float((lab != ignore_index).sum().item())
        gscale = 1.0 / n_valid if n_valid > 0 else 1.0
        hip = use_hip(h2) and h2.dtype == torch.bfloat16
        # gradients are produced in this pass: only when the caller runs with autograd on (an eval
        # forward under no_grad must neither compute dh nor touch W.main_grad)
        need_dh = ctx.needs_input_grad[0] and grad_enabled
        need_dw = ctx.needs_input_grad[1] and grad_enabled
        dh = torch.empty_like(h2) if need_dh else None
        mg = getattr(W, "main_grad", None) if need_dw else None
        dW = None
        if need_dw and mg is None:
            dW = torch.zeros(W.shape, dtype=torch.float32, device=W.device)
        losses = torch.empty(T, dtype=torch.float32, device=h2.device)
        buf = None
        # dh = dlogits . W through a cached W^T (TN GEMM layout, ~15 % faster): frozen heads keep one
        # copy, a trainable head (full FT) is re-transposed once per optimizer step
        from .linear import _TN_DW, accum_mm, transpose2d, transposed_weight

        WT = transposed_weight(W) if (need_dh and hip) else None
        for r0 in range(0, T, chunk_rows):
            r1 = min(T, r0 + chunk_rows)
            hc = h2[r0:r1]
            n = r1 - r0
            if buf is None or buf.shape[0] < n:
                buf = torch.empty(n, W.shape[0], dtype=h2.dtype, device=h2.device)
            logits = buf[:n]
            torch.mm(hc, W.t(), out=logits)
            labc = lab[r0:r1]
            if hip:
                losses[r0:r1] = ext().ce_fwd_bwd_(logits, labc.contiguous(), gscale, ignore_index)
                dlog = logits
            else:
                l, dlog = _ce_chunk_ref(logits, labc, gscale, ignore_index)
                losses[r0:r1] = l
            if need_dh:
                torch.mm(dlog, W if WT is None else WT.t(), out=dh[r0:r1])
            if need_dw:
                if mg is not None:
                    accum_mm(mg, dlog.t(), transpose2d(hc).t() if (hip and _TN_DW) else hc)
                else:
                    dW.addmm_(dlog.t().float(), hc.float())
        loss = losses.sum() * gscale
        ctx.save_for_backward(dh, dW)
        ctx.shp, ctx.wdtype = h.shape, W.dtype
        if mg is not None:
            from .linear import _GRAD_READY_HOOK

            if _GRAD_READY_HOOK is not None:
                _GRAD_READY_HOOK(W)
        return loss

    @staticmethod
    def backward(ctx, g):
        dh, dW = ctx.saved_tensors
        gh = None
        if dh is not None:
            gh = dh.mul_(g.to(dh.dtype)).view(ctx.shp)  # in place: dh is ours and used once
        gw = (dW * g).to(ctx.wdtype) if dW is not None else None
        return gh, gw, None, None, None, None, None


def fused_linear_cross_entropy(h: torch.Tensor, W: torch.Tensor, labels: torch.Tensor, chunk_rows: int = 4096,
                               ignore_index: int = -100, n_valid: float | None = None) -> torch.Tensor:
    """Mean CE over non-ignored labels. ``n_valid`` (optional) avoids a host sync per step; it is the
    normaliser (the loss is the sum over valid labels / n_valid) and may be fractional."""
    return _FusedLinearCE.apply(h, W, labels, chunk_rows, ignore_index, n_valid or 0, torch.is_grad_enabled())


def cross_entropy_reference(h, W, labels, ignore_index=-100):
    logits = (h.reshape(-1, h.shape[-1]).float() @ W.float().t())
    return F.cross_entropy(logits, labels.reshape(-1), ignore_index=ignore_index)
