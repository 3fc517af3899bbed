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

Both bf16 augmented weights (``AugProj``) and QLoRA NF4 weights (``NF4Proj``: dequantised per call
into the augmented / transposed operand) take this path.  The unfused composition
(``ops.linear.lora_linear`` / ``ops.nf4.qlora_linear`` + ``ops.activation.swiglu``) stays the
reference and the path for every other configuration (LoRA dropout, ranks other than 16 per segment,
optimizers without flat gradient buffers).
"""
from __future__ import annotations


import torch

from ._backend import ext, use_hip
from . import linear as _L
from .linear import _accum_xty, _grad_ready, _spare_cols, _tail, _wide, tail_product, tn_backward

_OFF = False  # True: the unfused composition (A/B by patching; profiles/r1_bench_fused_mlp*.log)


class AugProj:
    """A bf16 augmented projection (``ops.linear.AugWeight``) as seen by the fused MLP."""

    def __init__(self, aug, pair):
        self.aug, self.A, self.B, self.s = aug, pair.A, pair.B, float(pair.scale)
        self.N, self.K, self.R, self.Rp, self.nct = aug.N, aug.K, aug.R, aug.Rp, aug.nct

    def fwd_weight(self) -> torch.Tensor:  # [N, K+Rp] = [W | B 0]
        self.aug.refresh(self.A, self.B, self.s)
        return self.aug.big[:self.N]

    def fwd_tail(self) -> torch.Tensor:  # [Rp, K] = [s A ; 0]
        self.aug.refresh(self.A, self.B, self.s)
        return self.aug.big[self.N:, :self.K]

    def bwd_weight(self) -> torch.Tensor:  # [N+Rp, K] = [W ; s A ; 0] (TN view when enabled)
        self.aug.refresh(self.A, self.B, self.s)
        return self.aug.bwd_operand() if tn_backward() else self.aug.big[:, :self.K]

    def bwd_tail(self) -> torch.Tensor:  # [Rp, N] = B^T
        return self.aug.bwd_tail_operand(self.A, self.B, self.s)


class NF4Proj:
    """A QLoRA projection: the NF4 weight is dequantised per call straight into the augmented (forward)
    or transposed (backward) operand of ``ops.nf4``'s per-shape scratch; the rank-r tail operands live
    in ``ops.linear.TailOperands``."""

    def __init__(self, qw, tails, pair):
        from .nf4 import _QScratch

        self.qw, self.tails, self.A, self.B, self.s = qw, tails, pair.A, pair.B, float(pair.scale)
        self.N, self.K = qw.shape
        self.R, self.Rp, self.nct = tails.R, tails.Rp, tails.nct
        self.sc = _QScratch.get(self.N, self.K, self.Rp, pair.A.device)

    def fwd_weight(self) -> torch.Tensor:
        from .nf4 import _dequant_into

        N, K, R = self.N, self.K, self.R
        _dequant_into(self.qw, self.sc.fwd[:N, :K], False)
        self.sc.fwd[:N, K:K + R].copy_(self.B)
        return self.sc.fwd[:N]

    def fwd_tail(self) -> torch.Tensor:
        return self.tails.fwd_tail_operand(self.A, self.B, self.s)

    def bwd_weight(self) -> torch.Tensor:
        from .nf4 import _dequant_into

        N, R = self.N, self.R
        _dequant_into(self.qw, self.sc.bwdT[:, :N], True)
        self.sc.bwdT[:, N:N + R].copy_(self.fwd_tail()[:R].t())
        return self.sc.bwdT.t()

    def bwd_tail(self) -> torch.Tensor:
        return self.tails.bwd_tail_operand(self.A, self.B, self.s)


def fused_mlp_supported(x2: torch.Tensor, gu, dn, pair_gu, pair_down, p_gu: int, p_down: int,
                        training: bool) -> bool:
    """True when ``lora_mlp`` can run the fused path for this [T, d] input (padded row view) with the
    gate|up / down projections ``gu`` / ``dn`` (AugProj or NF4Proj)."""
    if _OFF or not use_hip(x2) or x2.dtype != torch.bfloat16 or x2.dim() != 2:
        return False
    if gu is None or dn is None:
        return False
    if training and (pair_gu.dropout > 0.0 or pair_down.dropout > 0.0):
        return False
    F = dn.K
    if not (gu.N == 2 * F and dn.N == gu.K and p_gu == gu.Rp and p_down == dn.Rp):
        return False
    if not (gu.R == 32 and dn.R == 16 and gu.Rp >= 32 and dn.Rp >= 16):
        return False
    blocks = pair_gu.blocks
    if not (blocks is not None and len(blocks) == 2 and tuple(blocks[0]) == (0, F, 0, 16)
            and tuple(blocks[1]) == (F, 2 * F, 16, 32)):
        return False
    for p in (pair_gu.A, pair_gu.B, pair_down.A, pair_down.B):
        mg = getattr(p, "main_grad", None)
        if mg is None or mg.dtype != torch.bfloat16:  # the fused weight-gradient kernel writes bf16
            return False
    if not _spare_cols(x2, gu.K, gu.Rp):
        return False
    if isinstance(gu, NF4Proj) or isinstance(dn, NF4Proj):
        from .nf4 import FUSED_MAX_ROWS

        q = gu if isinstance(gu, NF4Proj) else dn
        if (q.qw.block != 64 or gu.K % 64 or gu.N % 64 or dn.K % 64 or dn.N % 64
                or x2.shape[0] <= FUSED_MAX_ROWS):  # few rows: the fused NF4 GEMM path is faster
            return False
    # swiglu_bwd_wgrad's shape limits (csrc/kernels/swiglu_lora.hip): 512-column blocks
    return F % 512 == 0 and gu.Rp % 8 == 0


class _LoRAMLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, A_gu, B_gu, A_dn, B_dn, gu_p, dn_p):
        x2 = x.reshape(-1, x.shape[-1])
        T = x2.shape[0]
        K, N = gu_p.K, gu_p.N  # d, 2F
        F, d = dn_p.K, dn_p.N
        # 1. gate|up projection, LoRA folded in through x's spare columns
        tail_product(x2, K, gu_p.Rp, gu_p.fwd_tail(), gu_p.nct)
        gu = torch.mm(_wide(x2, K + gu_p.Rp), gu_p.fwd_weight().t())
        # 2. SwiGLU + s h A_down^T into h's spare columns
        h = ext().swiglu_fwd_lora(gu, dn_p.Rp, dn_p.fwd_tail(), dn_p.nct)
        # 3. down projection
        y = torch.empty(*x.shape[:-1], d, dtype=x.dtype, device=x.device)
        torch.mm(_wide(h, F + dn_p.Rp), dn_p.fwd_weight().t(), out=y.view(T, d))
        ctx.save_for_backward(x2, gu, h)
        ctx.params = (A_gu, B_gu, A_dn, B_dn)
        ctx.proj, ctx.shp = (gu_p, dn_p), x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        _L.join_wgrad_stream()  # the previous projection's side-stream weight gradients (ops.linear)
        x2, gu, h = ctx.saved_tensors
        A_gu, B_gu, A_dn, B_dn = ctx.params
        gu_p, dn_p = ctx.proj
        K, N = gu_p.K, gu_p.N
        F, d = dn_p.K, dn_p.N
        dy2 = dy.reshape(-1, dy.shape[-1])
        if not _spare_cols(dy2, d, dn_p.Rp):  # the producer gave no spare columns: pad here
            buf = torch.empty(dy2.shape[0], d + dn_p.Rp, dtype=dy2.dtype, device=dy2.device)
            buf[:, :d].copy_(dy2)
            dy2 = buf[:, :d]
        # 4. dy B_down into dy's spare columns, dh through the augmented (TN) operand
        tail_product(dy2, d, dn_p.Rp, dn_p.bwd_tail(), dn_p.nct)
        dyb_dn = _tail(dy2, d, dn_p.R)
        # 5. dB_down += dy^T (s h A_down^T)
        hta = _tail(h, F, dn_p.R)
        dh = torch.mm(_wide(dy2, d + dn_p.Rp), dn_p.bwd_weight())
        _accum_xty(B_dn.main_grad, dy2, hta, 1.0)
        _grad_ready(B_dn)
        # 6. SwiGLU backward + dgu B_gu + dB_gu + dA_down
        dgu = ext().swiglu_bwd_wgrad(dh, gu, gu_p.Rp, gu_p.bwd_tail(), _tail(x2, K, 32), dyb_dn, B_gu.main_grad,
                                     A_dn.main_grad, 1.0, dn_p.s)
        _grad_ready(B_gu)
        _grad_ready(A_dn)
        # 7. dx and dA_gu += s x^T (dgu B_gu)
        dgt = _tail(dgu, N, gu_p.R)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(_wide(dgu, N + gu_p.Rp), gu_p.bwd_weight()).view(ctx.shp)
        _accum_xty(A_gu.main_grad.t(), x2, dgt, gu_p.s)
        _grad_ready(A_gu)
        return dx, None, None, None, None, None, None


def lora_mlp(x: torch.Tensor, gu, dn) -> torch.Tensor:
    """Fused LoRA MLP (see module doc).  ``x``: the [T, d] column view of the post-norm buffer with
    ``gu.Rp`` spare columns; ``gu`` / ``dn``: AugProj or NF4Proj; call only when
    ``fused_mlp_supported`` holds."""
    return _LoRAMLPFn.apply(x, gu.A, gu.B, dn.A, dn.B, gu, dn)
