"""Projection GEMMs on the hand-written gfx950 kernels (csrc/kernels/gemm_nt.hip).

Every base GEMM of a LoRA / QLoRA step has the "NT" form ``C[T, n] = A[T, k] . B[n, k]^T`` with both
operands K-contiguous (ops/linear.py: the augmented forward ``[x | s x A^T] . [W | B]^T`` and the
input-gradient ``[dy | dy B] . [W ; s A]`` through the transposed frozen weight).  The hand-written
kernel is a persistent 256 x 256-tile MFMA GEMM with LDS-DMA staging (see the .hip header);
``ext().gemm_nt_config`` sets its launch configuration (persistent grid cap, tile order).
"""
from __future__ import annotations

import torch

from ._backend import ext, use_hip


# ---- routing of the projection GEMMs: hand-written kernel vs hipBLASLt ---------------------------------
# FTC_GEMM_NT: "0" -- hipBLASLt everywhere; "1" -- the gfx950 kernel wherever its contract holds;
# "auto" (default) -- the kernel only for the (N, K) shapes listed in NT_WINS, i.e. where an interleaved
# A/B on the MI355X measured it faster than hipBLASLt (tools/bench_gemm_nt.py, profiles/r4/gemm_nt.md),
# plus the RoPE-fused qkv projection for the shapes in ROPE_WINS (there the comparison is the library GEMM
# + the separate rope pass); "rope" -- only the RoPE-fused qkv projection.
NT_WINS: set[tuple[int, int]] = set()
ROPE_WINS: set[tuple[int, int]] = set()


def _nt_mode() -> str:
    import os

    return os.environ.get("FTC_GEMM_NT", "auto")


def mm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> bool:
    """``out = a @ b^T`` (a [M, K], b [N, K] row views, K contiguous) on the hand-written kernel when the
    routing policy picks it for this shape; False (nothing done) otherwise -- the caller then runs its
    library GEMM."""
    mode = _nt_mode()
    if mode in ("0", "rope") or not use_hip(a):
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
    if mode == "auto" and (b.shape[0], b.shape[1]) not in NT_WINS | ROPE_WINS:
        return False
    if not ext().gemm_nt_ok(out, a, b) or cos.shape[-1] != 64:
        return False
    ext().gemm_nt_rope_(out, a, b, cos, sin, pos, seq_len, n_rot)
    return True
