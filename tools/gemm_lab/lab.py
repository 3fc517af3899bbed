"""ctypes front-end of the GEMM lab library (``tools/gemm_lab/libgemm_lab.so``, built by ``build.sh``).

The hand-written projection (NT, with the fused RoPE epilogue) and weight-gradient (TN) GEMMs left the
package in round 6: neither beat hipBLASLt on a shipped shape (``profiles/r4/gemm_nt.md``,
``profiles/r5/gemm_nt.md``, ``profiles/r2/gemm_tn.md``), so ``_C.so`` carries only kernels that run on a
default path.  This module gives the lab benches and ``tests/test_gemm_lab.py`` the same call surface the
old ``_C`` bindings had (``gemm_nt_``, ``gemm_nt_ok``, ``gemm_nt_rope_``, ``gemm_nt_config``, ``gemm_tn_``,
``gemm_tn_ok``, ``gemm_tn_split_``), checking the same contracts on the host before any launch.
"""
from __future__ import annotations

import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libgemm_lab.so")

_P, _L, _I, _F = ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_float


class GemmLab:
    def __init__(self, path: str = LIB):
        if not os.path.exists(path):
            raise RuntimeError(f"{path} not built: bash tools/gemm_lab/build.sh")
        L = ctypes.CDLL(path)
        sig = {
            "ftc_gemm_nt_ok": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I, _I]),
            "ftc_gemm_nt": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _F, _F, _P]),
            "ftc_gemm_nt_config": (None, [_I, _I, _I]),
            "ftc_gemm_nt_rope": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I, _P, _P, _P, _I, _I, _P]),
            "ftc_gemm_tn_ok": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I]),
            "ftc_gemm_tn": (_I, [_P, _L, _P, _L, _P, _L, _I, _I, _I, _I, _F, _F, _P]),
            "ftc_gemm_tn_split": (_I, [_P, _L, _P, _L, _P, _I, _I, _I, _I, _P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        self.L = L

    @staticmethod
    def _stream():
        return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    @staticmethod
    def _rowview(*ts) -> bool:
        return all(t.is_cuda and t.dim() == 2 and t.stride(1) == 1 for t in ts)

    @staticmethod
    def _check(rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what}: launch failed / contract violated (rc {rc})")

    # ---- projection GEMM: c = alpha a b^T + beta c; a [M, K], b [N, K] bf16, c [M, N] bf16 / fp32
    def gemm_nt_ok(self, c, a, b) -> bool:
        if not self._rowview(a, b, c) or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
            return False
        if c.dtype not in (torch.bfloat16, torch.float32) or a.shape[1] != b.shape[1]:
            return False
        if c.shape[0] != a.shape[0] or c.shape[1] != b.shape[0]:
            return False
        return bool(self.L.ftc_gemm_nt_ok(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(),
                                          c.stride(0), int(c.dtype == torch.float32), a.shape[0], b.shape[0],
                                          a.shape[1]))

    def gemm_nt_(self, c, a, b, alpha: float = 1.0, beta: float = 0.0):
        if not self.gemm_nt_ok(c, a, b):
            raise RuntimeError("gemm_nt_: shapes / layouts outside the kernel contract (M, N % 256, K % 32, "
                               "bf16 row views a [M, K], b [N, K], c [M, N] bf16/fp32, 16-byte aligned)")
        self._check(self.L.ftc_gemm_nt(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(),
                                       c.stride(0), int(c.dtype == torch.float32), a.shape[0], b.shape[0],
                                       a.shape[1], alpha, beta, self._stream()), "gemm_nt_")

    def gemm_nt_rope_(self, c, a, b, cos, sin, positions, seq_len: int, rot_heads: int):
        if c.dtype != torch.bfloat16 or not self.gemm_nt_ok(c, a, b):
            raise RuntimeError("gemm_nt_rope_: GEMM contract (bf16 c)")
        if not (cos.dtype == sin.dtype == torch.float32 and cos.dim() == 2 and cos.shape[1] == 64
                and cos.is_contiguous() and sin.shape == cos.shape and sin.is_contiguous()):
            raise RuntimeError("gemm_nt_rope_: cos/sin [max_pos, 64] fp32 contiguous (head_dim 128)")
        pp = None
        if positions is not None:
            if positions.dtype != torch.int32 or positions.numel() != a.shape[0] or not positions.is_contiguous():
                raise RuntimeError("gemm_nt_rope_: positions [M] int32")
            pp = positions.data_ptr()
        elif not 0 < seq_len <= cos.shape[0]:
            raise RuntimeError("gemm_nt_rope_: seq_len within the table")
        self._check(self.L.ftc_gemm_nt_rope(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(),
                                            c.stride(0), a.shape[0], b.shape[0], a.shape[1], cos.data_ptr(),
                                            sin.data_ptr(), pp, int(seq_len), int(rot_heads), self._stream()),
                    "gemm_nt_rope_")

    def gemm_nt_config(self, grid_cap: int, group: int, xcc: int):
        self.L.ftc_gemm_nt_config(int(grid_cap), int(group), int(xcc))

    # ---- weight-gradient GEMM: c = beta c + alpha a^T b; a [K, M], b [K, N] bf16, c [M, N] bf16 / fp32
    def gemm_tn_ok(self, c, a, b) -> bool:
        if not self._rowview(a, b, c) or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
            return False
        if c.dtype not in (torch.bfloat16, torch.float32) or a.shape[0] != b.shape[0]:
            return False
        if c.shape[0] != a.shape[1] or c.shape[1] != b.shape[1]:
            return False
        return bool(self.L.ftc_gemm_tn_ok(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(),
                                          c.stride(0), a.shape[1], b.shape[1], a.shape[0]))

    def gemm_tn_(self, c, a, b, alpha: float = 1.0, beta: float = 0.0):
        if not self.gemm_tn_ok(c, a, b):
            raise RuntimeError("gemm_tn_: shapes / layouts outside the kernel contract (M, N % 256, K % 64, "
                               "bf16 row views a [K, M], b [K, N], c [M, N] bf16/fp32)")
        self._check(self.L.ftc_gemm_tn(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), c.data_ptr(),
                                       c.stride(0), int(c.dtype == torch.float32), a.shape[1], b.shape[1],
                                       a.shape[0], alpha, beta, self._stream()), "gemm_tn_")

    def gemm_tn_split_(self, parts, a, b):
        if not (parts.is_cuda and parts.dim() == 3 and parts.is_contiguous() and parts.dtype == torch.float32
                and self._rowview(a, b) and parts.shape[1] == a.shape[1] and parts.shape[2] == b.shape[1]
                and a.shape[0] == b.shape[0] and a.dtype == b.dtype == torch.bfloat16):
            raise RuntimeError("gemm_tn_split_: parts [S, M, N] fp32, a [K, M], b [K, N] bf16 row views")
        self._check(self.L.ftc_gemm_tn_split(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), parts.data_ptr(),
                                             a.shape[1], b.shape[1], a.shape[0], parts.shape[0], self._stream()),
                    "gemm_tn_split_ (shape outside the kernel contract: M, N % 256, K % (64 S))")


_lab: GemmLab | None = None


def load() -> GemmLab:
    global _lab
    if _lab is None:
        _lab = GemmLab()
    return _lab
