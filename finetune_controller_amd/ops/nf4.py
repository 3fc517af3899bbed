"""QLoRA: NF4 base weights (K8) and the LoRA linear over them.

``NF4Weight`` stores a frozen ``[out, in]`` weight as 4-bit NormalFloat codes (blocks of 64, one
absmax per block) with double quantisation of the absmax vector (uint8 codes + one fp32 scale per
256 absmaxes + a global offset): 0.5 + 1/64 + 4/16384 bytes per parameter, i.e. Mistral-7B's
7.2 B projection parameters take ≈3.7 GB instead of 14.5 GB.

Two GEMM paths, picked per call by shape:

* **fused** -- ``nf4_linear`` (``csrc/kernels/nf4_gemm.hip``): the NF4 decode happens in the MFMA
  kernel's B-operand staging (packed nibbles -> codebook -> x absmax -> bf16 LDS tile), so the bf16
  weight never exists in HBM.  Best when the weight stream dominates (few rows: decode, small
  micro-batches);
* **dequant + hipBLASLt** -- decode the whole weight into a transient bf16 buffer (one streaming
  kernel, ≈4.5 B/param of traffic) and run the library GEMM; best at training-sized M where the
  GEMM is compute bound and the decode is a few % of it.

The backward needs ``W`` again for ``dx = dy W`` and re-decodes it (nothing weight-sized is saved).
"""
from __future__ import annotations


import torch

from ._backend import ext, use_hip
from .linear import _mm_into, _spare_cols, _tail, _wide, direct_grad_params, lora_weight_grads, take_prefilled

NF4_CODE = torch.tensor([-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453, -0.28444138169288635,
                         -0.18477343022823334, -0.09105003625154495, 0.0, 0.07958029955625534, 0.16093020141124725,
                         0.24611230194568634, 0.33791524171829224, 0.44070982933044434, 0.5626170039176941,
                         0.7229568362236023, 1.0])

FUSED_MAX_ROWS = 128  # fused NF4 GEMM wins up to here (tools/bench_nf4.py, profiles/r1_bench_nf4.log)


class NF4Weight:
    def __init__(self, packed, absmax_q, absmax_scale, absmax_offset: float, shape, block=64, block2=256):
        self.packed, self.absmax_q, self.absmax_scale = packed, absmax_q, absmax_scale
        self.absmax_offset = float(absmax_offset)
        self.shape = tuple(shape)
        self.block, self.block2 = block, block2

    @property
    def device(self):
        return self.packed.device

    def nbytes(self) -> int:
        return self.packed.numel() + self.absmax_q.numel() + 4 * self.absmax_scale.numel()

    @classmethod
    @torch.no_grad()
    def quantize(cls, w: torch.Tensor, block: int = 64, block2: int = 256) -> "NF4Weight":
        rows, cols = w.shape
        flat = w.reshape(-1)
        if use_hip(w) and w.dtype == torch.bfloat16:
            packed, absmax = ext().nf4_quantize(flat.contiguous(), block)
        else:
            packed, absmax = _quantize_ref(flat, block)
        offset = float(absmax.mean().item())
        centered = absmax - offset
        nb2 = (absmax.numel() + block2 - 1) // block2
        pad = nb2 * block2 - absmax.numel()
        c2 = torch.nn.functional.pad(centered, (0, pad)).view(nb2, block2)
        scale2 = c2.abs().amax(1).clamp_min(1e-12)
        q2 = torch.round(c2 / scale2[:, None] * 127.0 + 128.0).clamp(0, 255).to(torch.uint8).reshape(-1)[: absmax.numel()]
        return cls(packed, q2.contiguous(), scale2.float().contiguous(), offset, (rows, cols), block, block2)

    def absmax(self) -> torch.Tensor:
        idx = torch.arange(self.absmax_q.numel(), device=self.absmax_q.device) // self.block2
        return self.absmax_offset + (self.absmax_q.float() - 128.0) / 127.0 * self.absmax_scale[idx]

    def dequantize(self, dtype=torch.bfloat16) -> torch.Tensor:
        if use_hip(self.packed):
            return ext().nf4_dequantize(self.packed, self.absmax_q, self.absmax_scale, self.absmax_offset,
                                        self.shape[0], self.shape[1], self.block, self.block2)
        return dequantize_reference(self).to(dtype)


def _quantize_ref(flat: torch.Tensor, block: int):
    x = flat.float().view(-1, block)
    absmax = x.abs().amax(1)
    xn = x / absmax.clamp_min(1e-30)[:, None]
    code = NF4_CODE.to(flat.device)
    q = (xn[..., None] - code).abs().argmin(-1).to(torch.uint8).reshape(-1)
    packed = (q[0::2] << 4) | q[1::2]
    return packed.contiguous(), absmax


def dequantize_reference(q: NF4Weight) -> torch.Tensor:
    code = NF4_CODE.to(q.packed.device)
    hi = (q.packed >> 4).long()
    lo = (q.packed & 0xF).long()
    vals = torch.stack([code[hi], code[lo]], dim=1).reshape(-1)
    am = q.absmax().repeat_interleave(q.block)
    return (vals * am).view(q.shape)


def nf4_matmul(x2: torch.Tensor, qw: NF4Weight) -> torch.Tensor:
    """x2 [M, K] @ W^T with W stored NF4 -> [M, N] (bf16)."""
    M = x2.shape[0]
    N, K = qw.shape
    if (use_hip(x2) and M <= FUSED_MAX_ROWS and K % 64 == 0 and N % 64 == 0 and qw.block == 64
            and getattr(ext(), "nf4_gemm_ready", lambda: False)()):
        return ext().nf4_linear(x2.contiguous(), qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, N,
                                qw.block, qw.block2)
    W = qw.dequantize(x2.dtype)
    return x2 @ W.t()


class _QScratch:
    """Per-shape bf16 scratch for the augmented QLoRA GEMMs (shared by every layer of that shape --
    layers run one after another on the stream, nothing here outlives a call):
    ``fwd [N+Rp, K+Rp] = [[W | B 0], [s A ; 0 | 0]]`` and ``bwdT [K, N+Rp] = [W^T | (s A)^T 0]``."""

    _cache: dict = {}

    def __init__(self, N, K, Rp, device):
        self.fwd = torch.zeros(N + Rp, K + Rp, dtype=torch.bfloat16, device=device)
        self.bwdT = torch.zeros(K, N + Rp, dtype=torch.bfloat16, device=device)
        self.Bp = torch.zeros(N, Rp, dtype=torch.bfloat16, device=device)

    @classmethod
    def get(cls, N, K, Rp, device):
        key = (N, K, Rp, str(device))
        sc = cls._cache.get(key)
        if sc is None:
            sc = cls._cache[key] = cls(N, K, Rp, device)
        return sc


def _dequant_into(qw: NF4Weight, out: torch.Tensor, transpose: bool):
    ext().nf4_dequantize_into(qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, out, qw.shape[0],
                              qw.shape[1], qw.block, qw.block2, transpose)


# (Removed in round 4: decoding the next NF4 operand on a side HIP stream under the current projection's
# GEMMs.  It engaged on every call (1,270 prefetches, 0 fallbacks) and measured -0.3 % on Mistral-7B QLoRA
# (37,181 / 37,229 / 37,240 vs 37,365 / 37,305 / 37,344 tok/s inline, profiles/r4/qlora_pf2/): the
# library's persistent GEMMs hold every CU, so the HBM-bound decode has nothing to run beside and only
# contends.  git history keeps it.)


# 0: the separate copy / scale kernels.  Mistral-7B QLoRA, interleaved on one box (profiles/r3/qlora_aug/):
# 439.88 / 439.70 ms fused vs 439.85 / 439.67 separate -- neutral (the 5 us copies it removes were hidden
# between launches); kept for the 4 fewer launches per projection call (hipGraph capture size)
_NF4_AUG = True  # W / B / s A in one decode launch (the three-launch path: tests / A/B by patching)


def _dequant_aug(qw: NF4Weight, out: torch.Tensor, transpose: bool, B, out_b, A, out_a, s: float):
    """``out`` = W (or W^T), ``out_b`` = B, ``out_a`` = s A (or (s A)^T) -- one kernel launch."""
    if not _NF4_AUG:
        _dequant_into(qw, out, transpose)
        if B is not None:
            out_b.copy_(B)
        if transpose:
            out_a.copy_((A * s).t())
        else:
            torch.mul(A, s, out=out_a)
        return
    ext().nf4_dequantize_aug(qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, out, qw.shape[0], qw.shape[1],
                             qw.block, qw.block2, transpose, B, out_b, A, out_a, float(s))


class _QLoRALinearFn(torch.autograd.Function):
    """y = x dequant(W)^T + s (x A^T) B^T with W in NF4.  On the GPU (LoRA present, padded producer
    buffers) the same augmented GEMMs as ops.linear run: the weight is dequantised straight into the
    augmented operand, and for the backward into its transposed (TN) form, so neither the rank-r
    read-modify-writes nor a separate transpose pass exist."""

    @staticmethod
    def forward(ctx, x, A, B, qw, scale, blocks, Rp, tails=None):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        N, K = qw.shape
        use_aug = (A is not None and Rp > 0 and use_hip(x2) and x2.dtype == torch.bfloat16
                   and x2.shape[0] > FUSED_MAX_ROWS and K % 64 == 0 and N % 64 == 0 and qw.block == 64
                   and _spare_cols(x2, K, Rp))
        xa = None
        if use_aug:
            R = A.shape[0]
            sc = _QScratch.get(N, K, Rp, x2.device)
            # W, B and s A into [[W | B 0], [s A ; 0 | 0]] in one launch (csrc/kernels/nf4.hip AugTail)
            _dequant_aug(qw, sc.fwd[:N, :K], False, B, sc.fwd[:N, K:K + R], A, sc.fwd[N:N + R, :K], scale)
            # the producer kernel (fused SwiGLU) may already have formed s x A^T in the spare columns
            if tails is None or not take_prefilled("fwd", x2, tails):
                _mm_into(x2, sc.fwd[N:, :K].t(), _tail(x2, K, Rp))
            xa = _tail(x2, K, R)  # s * x A^T
            y = torch.mm(_wide(x2, K + Rp), sc.fwd[:N].t())
        else:
            y = nf4_matmul(x2 if x2.is_contiguous() else x2.contiguous(), qw)
            if A is not None:
                xa = x2 @ A.t()
                y.addmm_(xa, B.t(), alpha=scale)
        ctx.save_for_backward(x2, A, B, xa)
        ctx.qw, ctx.scale, ctx.blocks, ctx.shp, ctx.Rp, ctx.aug_fwd = qw, scale, blocks, shp, Rp, use_aug
        ctx.tails = tails
        ctx.lora_params = direct_grad_params(A, B, blocks)
        return y if x.dim() == 2 else y.reshape(*shp[:-1], qw.shape[0]).clone()

    @staticmethod
    def backward(ctx, dy):
        x2, A, B, xa = ctx.saved_tensors
        s = ctx.scale
        qw = ctx.qw
        N, K = qw.shape
        Rp = ctx.Rp
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = dA = dB = dyb = None
        hip = use_hip(dy2) and dy2.dtype == torch.bfloat16 and qw.block == 64 and K % 64 == 0 and N % 64 == 0
        if ctx.needs_input_grad[0]:
            if hip and A is not None and Rp > 0 and _spare_cols(dy2, N, Rp):
                R = A.shape[0]
                sc = _QScratch.get(N, K, Rp, dy2.device)
                prefilled = ctx.tails is not None and take_prefilled("bwd", dy2, ctx.tails)
                # W^T, (s A)^T and (unless the producer formed dy B already) B for the tail product, one launch
                _dequant_aug(qw, sc.bwdT[:, :N], True, None if prefilled else B, None if prefilled else sc.Bp[:, :R],
                             A, sc.bwdT[:, N:N + R], s)
                if not prefilled:
                    _mm_into(dy2, sc.Bp, _tail(dy2, N, Rp))
                dyb = _tail(dy2, N, R)
                dx = torch.mm(_wide(dy2, N + Rp), sc.bwdT.t())
            elif hip:
                sc = _QScratch.get(N, K, 64, dy2.device)
                _dequant_into(qw, sc.bwdT[:, :N], True)  # TN operand even without LoRA spare columns
                dx = torch.mm(dy2, sc.bwdT[:, :N].t())
                if A is not None:
                    dyb = dy2 @ B
                    dx.addmm_(dyb, A, alpha=s)
            else:
                W = qw.dequantize(dy2.dtype)
                dx = dy2 @ W
                del W
                if A is not None:
                    dyb = dy2 @ B
                    dx.addmm_(dyb, A, alpha=s)
            dx = dx.view(ctx.shp)
        need_a, need_b = ctx.needs_input_grad[1], ctx.needs_input_grad[2]
        if A is not None and (need_a or need_b):
            if need_a and dyb is None:
                dyb = dy2 @ B
            dA, dB = lora_weight_grads(ctx.lora_params, dy2, xa, ctx.aug_fwd, dyb, x2, s, ctx.blocks, need_a, need_b)
        return dx, dA, dB, None, None, None, None, None


def qlora_linear(x, qw: NF4Weight, A=None, B=None, scale=1.0, blocks=None, pad: int = 0, tails=None):
    """``pad``: spare columns the producer of ``x`` (and of the output gradient) provides.  ``tails``
    (ops.linear.TailOperands): the producer kernels may form the rank-r tail products themselves."""
    return _QLoRALinearFn.apply(x, A, B, qw, scale, blocks, int(pad), tails)


@torch.no_grad()
def quantize_model_(model) -> int:
    """Replace every frozen projection weight of a Llama/Mistral model by an NF4Weight (in place).

    Returns bytes saved.  Embeddings, norms and lm_head stay bf16 (QLoRA convention)."""
    if model.cfg.family != "llama":
        raise ValueError("QLoRA quantisation is implemented for the Llama/Mistral trunk")
    saved = 0
    for layer in model.layers:
        for name, attr in (("qkv", "wqkv"), ("o", "wo"), ("gu", "wgu"), ("down", "wdown")):
            W = getattr(layer, attr)
            qw = NF4Weight.quantize(W.data.contiguous())
            layer.qweights[name] = qw
            saved += W.numel() * W.element_size() - qw.nbytes()
            setattr(layer, attr, torch.nn.Parameter(torch.empty(0, device=W.device, dtype=W.dtype), requires_grad=False))
            getattr(layer, "aug", {}).pop(name, None)  # drop the augmented bf16 buffer as well
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    return saved
