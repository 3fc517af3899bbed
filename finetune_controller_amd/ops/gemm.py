"""Projection GEMMs on the hand-written gfx950 kernels (csrc/kernels/gemm_nt.hip).

Every base GEMM of a LoRA / QLoRA step has the "NT" form ``C[T, n] = A[T, k] . B[n, k]^T`` with both
operands K-contiguous (ops/linear.py: the augmented forward ``[x | s x A^T] . [W | B]^T`` and the
input-gradient ``[dy | dy B] . [W ; s A]`` through the transposed frozen weight).  The weight operand is
frozen between optimizer steps, so it is stored once more in MFMA fragment order ("packed"): the
kernel then loads each 16 x 32 B fragment as one coalesced 1 KiB read straight into registers and only
the activation goes through LDS (the LDS traffic, not the matrix pipe, bounded the two-operand form).

Packed layout of B [N, K] (N % 32 == 0, K % 32 == 0): ``[N/32][K/32][2][64][8]`` -- for 32-row group g,
k-tile t, fragment f and lane l, element e is ``B[32 g + 8 ((l & 15) >> 2) + 4 f + (l & 3)][32 t + 8 (l >> 4) + e]``
(rows permuted inside the group so that each lane's two output tiles hold 8 consecutive columns).
"""
from __future__ import annotations

import torch

from ._backend import ext, use_hip


def pack_b_nt(b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """The packed fragment-order copy of ``b`` [N, K] (any strides; N, K multiples of 32) as a flat
    contiguous tensor of N * K elements."""
    N, K = b.shape
    if N % 32 or K % 32:
        raise ValueError(f"pack_b_nt needs N and K multiples of 32, got {tuple(b.shape)}")
    # rows r = 8 ih + 4 f + il of each 32-row group, k = 8 kc + e of each 32-wide tile
    v = b.reshape(N // 32, 4, 2, 4, K // 32, 4, 8)           # [g, ih, f, il, t, kc, e]
    v = v.permute(0, 4, 2, 5, 1, 3, 6)                       # [g, t, f, kc, ih, il, e]; lane = 16 kc + 4 ih + il
    if out is None:
        return v.contiguous().view(-1)
    out.view(N // 32, K // 32, 2, 4, 4, 4, 8).copy_(v)
    return out


def unpack_b_nt(bp: torch.Tensor, N: int, K: int) -> torch.Tensor:
    """Inverse of :func:`pack_b_nt` (tests)."""
    v = bp.view(N // 32, K // 32, 2, 4, 4, 4, 8)             # [g, t, f, kc, ih, il, e]
    return v.permute(0, 4, 2, 5, 1, 3, 6).reshape(N, K)      # [g, ih, f, il, t, kc, e]


def gemm_nt_packed(a: torch.Tensor, bp: torch.Tensor, N: int, out: torch.Tensor | None = None,
                   alpha: float = 1.0, beta: float = 0.0) -> torch.Tensor:
    """``out = alpha a . B^T + beta out`` with B given packed; HIP kernel on the GPU, torch elsewhere."""
    K = a.shape[1]
    if out is None:
        out = torch.empty(a.shape[0], N, dtype=a.dtype, device=a.device)
        beta = 0.0
    if use_hip(a) and ext().gemm_nt_pb_ok(out, a, bp, N, K):
        ext().gemm_nt_pb_(out, a, bp, N, K, float(alpha), float(beta))
        return out
    ref = torch.mm(a.float(), unpack_b_nt(bp, N, K).float().t()) * alpha
    if beta != 0.0:
        ref += beta * out.float()
    out.copy_(ref)
    return out


# ---- routing of the projection GEMMs: hand-written kernel vs hipBLASLt ---------------------------------
# FTC_GEMM_NT: "0" -- hipBLASLt everywhere; "1" -- the gfx950 kernel wherever its contract holds;
# "auto" (default) -- the kernel only for the (N, K) shapes listed in NT_WINS, i.e. where an interleaved
# A/B on the MI355X measured it faster than hipBLASLt (tools/bench_gemm_nt.py, profiles/r3/gemm_nt.md).
NT_WINS: set[tuple[int, int]] = set()


def _nt_mode() -> str:
    import os

    return os.environ.get("FTC_GEMM_NT", "auto")


def mm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> bool:
    """``out = a @ b^T`` (a [M, K], b [N, K] row views, K contiguous) on the hand-written kernel when the
    routing policy picks it for this shape; False (nothing done) otherwise -- the caller then runs its
    library GEMM."""
    mode = _nt_mode()
    if mode == "0" or not use_hip(a):
        return False
    if mode != "1" and (b.shape[0], b.shape[1]) not in NT_WINS:
        return False
    if not ext().gemm_nt_ok(out, a, b):
        return False
    ext().gemm_nt_(out, a, b, 1.0, 0.0)
    return True


def mm(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """``a @ b`` for the projection GEMMs: when ``b`` is the transpose of a K-contiguous [N, K] matrix
    (a weight ``W.t()`` or the TN copy's view) the routing policy may send it to the hand-written
    kernel; otherwise / on fallback ``torch.mm`` (hipBLASLt)."""
    if out is None:
        out = torch.empty(a.shape[0], b.shape[1], dtype=a.dtype, device=a.device)
    bt = b.t()
    if bt.dim() == 2 and bt.stride(1) == 1 and mm_nt(a, bt, out):
        return out
    return torch.mm(a, b, out=out)


def rope_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor, rope: tuple) -> bool:
    """``out = rope(a @ b^T)`` with the rotation in the hand-written kernel's epilogue (head_dim 128), when
    the routing policy picks the kernel for this shape; False (nothing done) otherwise."""
    cos, sin, pos, seq_len, n_rot, hd = rope[:6]
    mode = _nt_mode()
    if hd != 128 or mode == "0" or not use_hip(a) or out.dtype != torch.bfloat16:
        return False
    if mode != "1" and (b.shape[0], b.shape[1]) not in NT_WINS:
        return False
    if not ext().gemm_nt_ok(out, a, b) or cos.shape[-1] != 64:
        return False
    ext().gemm_nt_rope_(out, a, b, cos, sin, pos, seq_len, n_rot)
    return True
