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

**Augmented GEMMs** (MI355X path, ``AugWeight``).  The rank-r update folded into the big GEMMs
instead of a read-modify-write of the [T, N] output (and of the [T, K] input gradient):

* forward   ``y  = [x | s x A^T] . [W | B]^T``       -- one GEMM with K + Rp columns
* backward  ``dx = [dy | dy B] . [W ; s A]``          -- one GEMM with N + Rp rows

One buffer ``big [N+Rp, K+Rp]`` (Rp = R rounded up to the 64-wide GEMM K-tile: hipBLASLt's
K-tail handling cost more than the rank update saved) holds W in ``big[:N, :K]`` (the frozen
Parameter is a view of it), ``[B | 0]`` in ``big[:N, K:]`` and ``[s A ; 0]`` in ``big[N:, :K]``
(refreshed from the trainable A/B each call).  The producers of ``x`` (RMSNorm, flash attention,
SwiGLU) and of ``dy`` (flash backward, SwiGLU backward) write into row-padded buffers, so
``s x A^T`` / ``dy B`` (and the zero pad columns) land in the spare columns and the augmented
operands are plain strided views -- no concatenation copies.  When an operand has no spare
columns the two-GEMM path runs instead.
"""
from __future__ import annotations

import os
import struct
import weakref

import torch

from ._backend import ext, use_hip

_GRAD_READY_HOOK = None  # set by parallel.ddp to learn when a main_grad was written

# Bumped by optimizers that rewrite parameters in place behind autograd's back (the flat AdamW kernel
# writes param_flat directly, which moves no version counter): AugWeight re-copies A/B then.
_PARAM_GENERATION = [0]


def bump_param_generation():
    _PARAM_GENERATION[0] += 1


def _refresh_key(A: torch.Tensor, B: torch.Tensor, scale: float) -> tuple:
    return (_PARAM_GENERATION[0], A._version, B._version, A.data_ptr(), B.data_ptr(), float(scale))


# ---- batched operand refresh.  After an optimizer step every augmented projection needs its A / B
# copies (s A, B, and the transposed s A^T / B^T where kept) refreshed: ~16 small copy / scale launches
# per layer.  The first refresh of a parameter generation refreshes EVERY bound operand set in one
# launch (csrc/kernels/elementwise.hip ``copy2d_batched``); the later calls find their key current.
_BATCH_REFRESH = True
_BOUND: list = []  # weakrefs to AugWeight / TailOperands bound to their (A, B, scale)
_JOB_TABLES: dict = {}  # packed job table bytes -> device int64 tensor (addresses are stable per model)


class _Refreshable:
    _key = None
    _bind = None

    def refresh(self, A: torch.Tensor, B: torch.Tensor, scale: float):
        key = _refresh_key(A, B, scale)
        if key == self._key:
            return
        if self._bind is None:
            self._bind = (A, B, float(scale))
            _BOUND.append(weakref.ref(self))
        bound = self._bind[0] is A and self._bind[1] is B and self._bind[2] == float(scale)
        if not (_BATCH_REFRESH and bound and refresh_bound()):
            self._refresh_now(A, B, scale)
            self._key = key

    def _refresh_now(self, A, B, scale):
        for dst, src, sc in self._copy_jobs(A, B, float(scale)):
            if sc == 1.0:
                dst.copy_(src)
            else:
                torch.mul(src, sc, out=dst)

    def _copy_jobs(self, A, B, scale) -> list:
        raise NotImplementedError


def _pack_job(dst: torch.Tensor, src: torch.Tensor, scale: float) -> bytes:
    if dst.stride(1) != 1:  # orient so the destination row is contiguous (coalesced stores)
        dst, src = dst.t(), src.t()
    rows, cols = dst.shape
    return struct.pack("<qqqqqqiifi", src.data_ptr(), dst.data_ptr(), src.stride(0), src.stride(1), dst.stride(0),
                       dst.stride(1), rows, cols, float(scale), 0)


def refresh_bound() -> bool:
    """Refresh every bound operand set whose key is stale in one launch.  False (nothing done) when
    any of them cannot take the HIP path; the caller then refreshes itself the plain way."""
    stale, alive = [], []
    for r in _BOUND:
        o = r()
        if o is None:
            continue
        alive.append(r)
        A, B, sc = o._bind
        k = _refresh_key(A, B, sc)
        if k != o._key:
            stale.append((o, k))
    _BOUND[:] = alive
    jobs = []
    for o, _ in stale:
        A, B, sc = o._bind
        for dst, src, js in o._copy_jobs(A, B, sc):
            if not (use_hip(dst) and dst.dtype == src.dtype == torch.bfloat16 and dst.device == src.device
                    and dst.dim() == 2 and dst.shape == src.shape and 1 in dst.stride() and dst.numel() > 0):
                return False
            jobs.append((dst, src, js))
    if not jobs:
        return True
    if not hasattr(ext(), "copy2d_batched_"):
        return False
    dev = jobs[0][0].device
    if any(d.device != dev for d, _, _ in jobs):
        return False
    blob = b"".join(_pack_job(*j) for j in jobs)
    table = _JOB_TABLES.get(blob)
    if table is None:
        if len(_JOB_TABLES) > 8:
            _JOB_TABLES.clear()
        import numpy as np

        table = torch.from_numpy(np.frombuffer(blob, dtype=np.int64).copy()).to(dev)
        _JOB_TABLES[blob] = table
    for i in range(0, len(jobs), 65535):
        n = min(65535, len(jobs) - i)
        ext().copy2d_batched_(table[i * 8:(i + n) * 8], n, max(d.numel() for d, _, _ in jobs[i:i + n]))
    for o, k in stale:
        o._key = k
    return True


def set_grad_ready_hook(fn):
    global _GRAD_READY_HOOK
    _GRAD_READY_HOOK = fn


def _grad_ready(p):
    if _GRAD_READY_HOOK is not None:
        _GRAD_READY_HOOK(p)


# ---- weight gradients on a side stream (full fine-tuning).  dW += dy^T x is off the backward's critical
# path (nothing downstream reads it until the optimizer), so it can run on its own HIP stream beside the
# input-gradient GEMM, the attention / SwiGLU / norm backward kernels and the transposes: the two queues'
# workgroups fill each other's tail waves (the qkv dW GEMM is 1.5 waves of 256x256 tiles on 256 CUs, the
# down dW 3.5) and HBM-bound kernels run under matrix-bound ones.  Ordering, by construction:
#   * the side stream waits for the main stream before each dW (dy and x are final);
#   * the NEXT linear backward (and ``join_wgrad_stream``, called by the trainer after backward) makes
#     the main stream wait for the previous dW: an input gradient that autograd later accumulates into
#     in place (the residual stream's gradient is the down / o projections' dy) is not touched before
#     the dW that reads it has finished -- every such accumulation happens after at least one more
#     projection backward;
#   * dy and x stay referenced until that join (no early allocator reuse, no record_stream: a
#     record_stream'ed block is withheld from the main stream's pool until an event query says the side
#     stream is done, which at full-FT memory pressure (218 GB of 288) ended in cache flushes and re-
#     allocations -- 3x slower steps); the transposed x lives in one persistent side-stream buffer;
#   * gradient buckets (parallel.ddp) are launched from the side stream after it has waited for main.
# ``FTC_DW_STREAM`` (default on; ``0`` = every dW on the main stream) / ``set_wgrad_stream``.  Measured on
# Llama-3-8B full FT, interleaved on one box (profiles/r3/dw_side/): with the dW issued BEFORE the input-
# gradient GEMM (the two run concurrently) 702.1 / 700.8 ms vs 705.2 / 705.9 ms serial (+0.5 %); issued
# after it (so only the following kernels overlap) it had measured 700.0 / 700.4 vs 696.8 / 697.0 (-0.5 %).
_DW_STREAM = os.environ.get("FTC_DW_STREAM", "1") != "0"
_DW_SIDE: dict = {}
_DW_PENDING: list = []  # [event] of the last side-stream dW not yet waited for by the main stream


def set_wgrad_stream(on: bool) -> None:
    global _DW_STREAM
    join_wgrad_stream()
    _DW_STREAM = bool(on)


def wgrad_stream_active() -> bool:
    return _DW_STREAM


def _wgrad_side(device) -> torch.cuda.Stream:
    st = _DW_SIDE.get(device)
    if st is None:
        st = _DW_SIDE[device] = torch.cuda.Stream(device=device)
    return st


def join_wgrad_stream() -> None:
    """Order the current stream after every weight gradient issued on the side stream so far (and drop
    the operand references held for it)."""
    if _DW_PENDING:
        ev, dev = _DW_PENDING[0][:2]
        torch.cuda.current_stream(dev).wait_event(ev)
        _DW_PENDING.clear()


# ``FTC_DW_GATE`` (VERDICT r5 Next #6): the HBM-bound backward kernels (SwiGLU, RMSNorm, flash attention
# backward) wait for the in-flight side-stream dW before they launch, so a dW GEMM overlaps only the input-
# gradient GEMM it was issued beside, never a stream kernel it would starve (swiglu_bwd 1.85 ms/call under
# overlap vs 0.41 serial, profiles/r5/kernel_tables/full_ft.md).
_DW_GATE = os.environ.get("FTC_DW_GATE", "0") == "1"


def set_wgrad_gate(on: bool) -> None:
    global _DW_GATE
    _DW_GATE = bool(on)


def gate_wgrad_stream() -> None:
    """Called by the HBM-bound backward kernels before they launch: join the side-stream dW when gated."""
    if _DW_GATE:
        join_wgrad_stream()


def wgrad_launch_stream():
    """The stream gradient collectives must be enqueued on (parallel.ddp): the side stream, after it has
    waited for the main stream, while side-stream weight gradients are in flight; else None (current)."""
    if not _DW_PENDING:
        return None
    dev = _DW_PENDING[0][1]
    side = _wgrad_side(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    return side


_DW_XT: dict = {}  # device -> flat bf16 buffer for the transposed activation (side stream only)


def _wgrad_on_side(mg: torch.Tensor, dy2: torch.Tensor, x2: torch.Tensor, tn_dw: bool, beta: float = 1.0):
    dev = dy2.device
    join_wgrad_stream()  # (already joined by the caller's backward; keeps one dW in flight at most)
    main = torch.cuda.current_stream(dev)
    side = _wgrad_side(dev)
    xt = None
    if tn_dw:
        n = x2.shape[0] * x2.shape[1]
        buf = _DW_XT.get(dev)
        if buf is None or buf.numel() < n or buf.dtype != x2.dtype:
            buf = _DW_XT[dev] = torch.empty(n, dtype=x2.dtype, device=dev)
        xt = buf[:n].view(x2.shape[1], x2.shape[0])
    side.wait_stream(main)
    with torch.cuda.stream(side):
        if xt is not None:
            transpose2d(x2, xt)
            wgrad_mm(mg, dy2.t(), xt.t(), beta=beta)
        else:
            wgrad_mm(mg, dy2.t(), x2, beta=beta)
        ev = torch.cuda.Event()
        ev.record(side)
    _DW_PENDING[:] = [(ev, dev, dy2, x2)]


# (Removed: LoRA adapter weight gradients on the side stream under the input-gradient GEMM --
# 35,213 / 35,138 vs 35,562 / 35,473 tok/s serial, profiles/r3/lora_wg/: the 30 us rank-r kernels stretch
# the big GEMMs they share the CUs with more than their own time.)


def _mask_blocks(dB: torch.Tensor, blocks):
    """Zero everything outside the diagonal blocks [(row0,row1,col0,col1), ...]."""
    if blocks is None:
        return dB
    out = torch.zeros_like(dB)
    for r0, r1, c0, c1 in blocks:
        out[r0:r1, c0:c1] = dB[r0:r1, c0:c1]
    return out


def _spare_cols(t: torch.Tensor, width: int, extra: int) -> bool:
    """True if the 2-D row view ``t[:, :width]`` has ``extra`` writable columns after it in every row."""
    if t.dim() != 2 or t.stride(1) != 1 or t.stride(0) < width + extra or extra <= 0:
        return False
    need = t.storage_offset() + (t.shape[0] - 1) * t.stride(0) + width + extra
    return t.untyped_storage().nbytes() >= need * t.element_size()


def _tail(t: torch.Tensor, width: int, extra: int) -> torch.Tensor:
    return t.as_strided((t.shape[0], extra), (t.stride(0), 1), t.storage_offset() + width)


# PyTorch TunableOp assumes ldc == n for GEMM outputs: under it the spare-column products go through
# a contiguous temporary (two tiny copies per call) instead of being written in place
_TUNABLEOP = os.environ.get("PYTORCH_TUNABLEOP_ENABLED", "0") == "1"
_TN_BWD = os.environ.get("FTC_TN_BWD", "1") != "0"  # transposed frozen-weight copies for backward GEMMs


def set_tn_backward(on: bool) -> None:
    """Enable / disable the W^T copies of the TN backward GEMMs (+2 B per weight element of HBM);
    the trainer turns them off when the copies would not fit next to the model (e.g. 70B bf16)."""
    global _TN_BWD
    _TN_BWD = bool(on) and os.environ.get("FTC_TN_BWD", "1") != "0"


def tn_backward() -> bool:
    return _TN_BWD


class FrozenTransposed:
    """Cache of ``W^T`` (contiguous) for frozen 2-D weights used as the right operand of ``x @ W`` in a
    backward pass (TN layout, see AugWeight.bwd_operand).  Keyed by the parameter; rebuilt when the
    parameter's version counter moves (in-place loads / init)."""

    def __init__(self):
        self._c: dict[int, tuple] = {}

    def get(self, W: torch.Tensor) -> torch.Tensor:
        key = id(W)
        hit = self._c.get(key)
        if hit is not None and hit[0] == W.data_ptr() and hit[1] == W._version:
            return hit[2]
        WT = W.detach().t().contiguous()
        self._c[key] = (W.data_ptr(), W._version, WT)
        return WT

    def clear(self):
        self._c.clear()


frozen_t = FrozenTransposed()


class TrainableTransposed(FrozenTransposed):
    """``W^T`` copies of TRAINABLE weights (full fine-tuning) for the TN backward GEMM: the flat AdamW
    kernel rewrites ``param_flat`` without moving version counters, so the key also carries the
    optimizer generation -- one transpose per weight per step (+2 B/param of HBM), shared by every
    micro-batch of the step."""

    def get(self, W: torch.Tensor) -> torch.Tensor:
        key = id(W)
        hit = self._c.get(key)
        tag = (W.data_ptr(), W._version, _PARAM_GENERATION[0])
        if hit is not None and hit[0] == tag:
            return hit[2]
        old = hit[2] if hit is not None else None
        WT = transpose2d(W.detach(), out=old if old is not None and old.shape == (W.shape[1], W.shape[0]) else None)
        self._c[key] = (tag, None, WT)
        return WT


param_t = TrainableTransposed()
_TN_DW = True  # weight gradients with the activation transposed (14-24 % faster, profiles/r1_dw_gemm_layouts.log)


def transpose2d(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Contiguous ``x^T`` of a 2-D row view: the HIP LDS-tiled transpose on GPU (csrc/kernels/transpose.hip)."""
    if (use_hip(x) and x.dtype == torch.bfloat16 and x.stride(1) == 1 and x.shape[0] % 8 == 0
            and x.shape[1] % 8 == 0 and x.stride(0) % 8 == 0):
        return ext().transpose2d(x, out)
    if out is not None:
        return out.copy_(x.t())
    return x.t().contiguous()


def transposed_weight(W: torch.Tensor) -> torch.Tensor | None:
    """W^T for the TN backward GEMM dx = dy W (None when the TN path is off or not on the HIP backend)."""
    if not (_TN_BWD and use_hip(W) and W.dim() == 2):
        return None
    return (param_t if W.requires_grad else frozen_t).get(W)


def accum_mm(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, alpha: float = 1.0,
             beta: float = 1.0) -> torch.Tensor:
    """``out = beta * out + alpha * a @ b`` (beta 0: ``out``'s old values are ignored, NaNs included).
    ``out`` may be wider than the operands (fp32 gradient buffer with bf16 activations): on the GPU one
    GEMM with bf16 A/B and an fp32 C/D (in place), so the accumulation never rounds to bf16."""
    if out.dtype == a.dtype:
        return out.addmm_(a, b, beta=beta, alpha=alpha)
    if a.is_cuda:
        return torch.addmm(out, a, b, beta=beta, alpha=alpha, out_dtype=out.dtype, out=out)
    return out.addmm_(a.to(out.dtype), b.to(out.dtype), beta=beta, alpha=alpha)


# ---- split-K weight gradients (full fine-tuning).  The weight-gradient GEMMs reduce over all T tokens
# of the micro-batch; two of the Llama-3-8B shapes leave the last wave of 256 x 256 tiles half empty on
# 256 CUs (qkv: 384 tiles = 1.5 waves, down: 896 = 3.5).  Split along the tokens into S slices so that
# S x tiles is a whole number of waves: ONE batched hipBLASLt GEMM writes the S fp32 partials, one HIP
# pass (csrc/kernels/elementwise.hip splitk_sum_kernel) folds them into the gradient (beta C + sum).
# FTC_DW_SPLIT: "auto" (default: the measured winning shapes), "0" off, or a fixed S.
_DW_SPLIT = os.environ.get("FTC_DW_SPLIT", "auto")  # full FT +0.9 % (profiles/r4/dw_split/full_ab)
_WAVE = 256  # workgroups per wave: one 256 x 256 tile per CU


def dw_splits(M: int, N: int, K: int, mode: str | None = None) -> int:
    """Token slices for the weight gradient of an [M, N] weight reduced over K tokens (1 = no split)."""
    mode = _DW_SPLIT if mode is None else mode
    if mode == "0":
        return 1
    if mode != "auto":
        s = int(mode)
        return s if s > 1 and K % (64 * s) == 0 else 1
    # measured (profiles/r4/dw_split/): only the wide-input shape gains -- down dW [4096, 14336] 1.90 ->
    # 1.68 ms (hipBLASLt's 3.5 waves of 256 x 256 tiles -> 7); qkv [6144, 4096] runs 1,240 TF/s unsplit
    # (the library's own tiling is not 1.5 waves there) and loses 3 % split; o / gate-up are whole waves
    tiles = -(-M // 256) * -(-N // 256)
    if N < 2 * M or tiles % _WAVE == 0 or tiles > 8 * _WAVE:
        return 1
    for s in (2, 4):
        if (tiles * s) % _WAVE == 0 and K % (64 * s) == 0:
            return s
    return 1


def wgrad_mm(out: torch.Tensor, a: torch.Tensor, b: torch.Tensor, beta: float = 1.0) -> torch.Tensor:
    """``out = beta * out + a @ b`` for a weight gradient (``a`` = dy^T [M, T], ``b`` = x [T, N], any
    strides): split along T when ``dw_splits`` says so, else ``accum_mm``."""
    M, K = a.shape
    N = b.shape[1]
    s = dw_splits(M, N, K) if (use_hip(a) and out.stride(1) == 1) else 1
    if s == 1:
        return accum_mm(out, a, b, beta=beta)
    k = K // s
    A = a.as_strided((s, M, k), (k * a.stride(1), a.stride(0), a.stride(1)))
    B = b.as_strided((s, k, N), (k * b.stride(0), b.stride(0), b.stride(1)))
    parts = _dw_parts(a.device, s, M, N)
    torch.bmm(A, B, out_dtype=torch.float32, out=parts)
    ext().splitk_sum_(out, parts, float(beta))
    return out


def _dw_parts(device, s: int, M: int, N: int) -> torch.Tensor:
    """fp32 split-K partials, from the caching allocator per call: the block goes back to the pool of the
    stream it was taken on after the fold (no per-stream buffer pinned for the life of the process;
    ``utils.memplan`` counts one per dW stream in the full-FT peak)."""
    return torch.empty((s, M, N), dtype=torch.float32, device=device)


# ---- first-write weight gradients (full fine-tuning).  Zeroing the 16 GB gradient buffer of Llama-3-8B
# costs 2.8 ms per step; the projection weights (7 of its 8 B parameters) are each written by exactly one
# beta = 1 GEMM per micro-batch, so the optimizer skips their slices (FlatAdamW.zero_grad) and marks them
# "fresh": their first GEMM of the step runs with beta = 0 instead.  A weight joins the set only after a
# step in which it was zeroed and written by that GEMM; one that a step leaves fresh (never written) is
# zeroed by ``flush_fresh`` before the gradients are used.  Default on (``_FIRST_WRITE = False``: zero
# the whole buffer): Llama-3-8B full FT, interleaved on one box (profiles/r3/first_write/), 690.1 / 692.0 ms
# vs 693.7 / 694.4 ms/step (+0.4 %).
_FIRST_WRITE = True
# id(param) -> weakref(param): weights only a projection GEMM writes.  Entries are identity-checked (a dead
# parameter's id can be reused by a new tensor of another trainer) and hold no reference to the gradient
# buffer (a main_grad view would keep a whole flat fp32 buffer alive after its optimizer is gone)
_GRAD_OWNED: dict = {}
_GRAD_FRESH: set = set()  # ids whose main_grad still holds last step's values


def set_first_write(on: bool) -> None:
    global _FIRST_WRITE
    _FIRST_WRITE = bool(on)
    _GRAD_OWNED.clear()
    _GRAD_FRESH.clear()


def reset_grad_owned() -> None:
    """Forget every registered weight (a new optimizer re-homes the gradients: each weight is zeroed and
    written once more before it may skip zeroing again)."""
    _GRAD_OWNED.clear()
    _GRAD_FRESH.clear()


def is_grad_owned(p) -> bool:
    e = _GRAD_OWNED.get(id(p)) if _FIRST_WRITE else None
    return e is not None and e() is p


def mark_fresh(ids) -> None:
    _GRAD_FRESH.update(ids)


def take_fresh(p, mg: torch.Tensor) -> float:
    """beta for the projection GEMM that writes ``p``'s gradient now: 0 on its first write of the step
    when the optimizer skipped zeroing it, else 1 (and ``p`` is registered for the next step)."""
    if not _FIRST_WRITE or (mg.is_cuda and torch.cuda.is_current_stream_capturing()):
        return 1.0
    pid = id(p)
    e = _GRAD_OWNED.get(pid)
    if e is None or e() is not p:  # first sight of this parameter: its gradient was zeroed this step
        _GRAD_OWNED[pid] = weakref.ref(p)
        _GRAD_FRESH.discard(pid)
        return 1.0
    if pid in _GRAD_FRESH:
        _GRAD_FRESH.discard(pid)
        return 0.0
    return 1.0


def flush_fresh() -> None:
    """Zero the gradient of every skipped weight that this step did not write (call before reading them:
    the optimizers and the gradient bucketer do, see ``gradients_final``)."""
    while _GRAD_FRESH:
        e = _GRAD_OWNED.get(_GRAD_FRESH.pop())
        p = e() if e is not None else None
        mg = getattr(p, "main_grad", None) if p is not None else None
        if mg is not None:
            mg.zero_()


def gradients_final() -> None:
    """Make the gradient buffer safe to read on the current stream: join the side-stream weight
    gradients and zero the skipped weights this step never wrote.  Cheap no-ops when nothing is pending;
    called at the top of every optimizer step / gradient-norm / bucket-finish, so a plain
    ``zero_grad(); loss.backward(); step()`` loop is correct without trainer help."""
    join_wgrad_stream()
    flush_fresh()


def _mm_into(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor):
    if _TUNABLEOP:
        out.copy_(torch.mm(a, b))
    else:
        torch.mm(a, b, out=out)


# Tail products already formed by the producer kernel of an operand (one slot per direction; every
# augmented GEMM call of that direction consumes the slot, so a mark never outlives its consumer).
_PREFILLED: dict[str, tuple] = {}


def _operand_key(t: torch.Tensor, aug) -> tuple:
    return (t.data_ptr(), t.stride(0), t.shape[0], id(aug), aug._key)


def mark_prefilled(direction: str, t: torch.Tensor, aug) -> None:
    """``t`` ([T, width] row view) already holds the tail product of ``aug`` in its spare columns."""
    _PREFILLED[direction] = _operand_key(t, aug)


def take_prefilled(direction: str, t: torch.Tensor, aug) -> bool:
    v = _PREFILLED.pop(direction, None)
    return v is not None and v == _operand_key(t, aug)


class TailOperands(_Refreshable):
    """Stand-alone tail operands for a projection whose weight is not an ``AugWeight`` (QLoRA: the NF4
    weight is dequantised per call into a shared scratch): ``[s A ; 0]`` as [Rp, K] and ``B^T`` as
    [Rp, N], refreshed once per optimizer generation -- the same interface as AugWeight's
    ``fwd_tail_operand`` / ``bwd_tail_operand``."""

    def __init__(self, N: int, K: int, R: int, Rp: int, device=None, dtype=torch.bfloat16):
        self.N, self.K, self.R, self.Rp = N, K, R, Rp
        self.fwd = torch.zeros(Rp, K, device=device, dtype=dtype)
        self.bt = torch.zeros(Rp, N, device=device, dtype=dtype)
        self._key = None

    @property
    def nct(self) -> int:
        return -(-self.R // 16)

    def _copy_jobs(self, A, B, scale) -> list:
        return [(self.fwd[:self.R], A, scale), (self.bt[:self.R], B.t(), 1.0)]

    def fwd_tail_operand(self, A, B, scale):
        self.refresh(A, B, scale)
        return self.fwd

    def bwd_tail_operand(self, A, B, scale):
        self.refresh(A, B, scale)
        return self.bt


class LoRATail:
    """What a producer kernel needs to form the LoRA tail of its consumer's augmented GEMM."""

    __slots__ = ("aug", "A", "B", "scale", "split")

    def __init__(self, aug, A, B, scale, blocks=None):
        self.aug, self.A, self.B, self.scale = aug, A, B, float(scale)
        # two-segment block-diagonal B (packed gate|up) whose halves own 16-aligned tail column
        # ranges: the producer feeds each half of its output only to its own tail tiles
        R = aug.R
        self.split = bool(blocks is not None and len(blocks) == 2 and R % 32 == 0
                          and tuple(blocks[0][2:]) == (0, R // 2) and tuple(blocks[1][2:]) == (R // 2, R)
                          and blocks[0][0] == 0 and blocks[0][1] == blocks[1][0] == aug.N // 2
                          and blocks[1][1] == aug.N)


_HIP_TAIL = True  # False: hipBLASLt for the skinny tail GEMMs (A/B by patching; profiles/r1_tail_gemm_ab.log)
_HIP_TAIL_MAX_NCT = 2  # widest tail (in 16-column tiles) the HIP kernel takes


def tail_product(x2: torch.Tensor, width: int, Rp: int, operand: torch.Tensor, nct: int) -> None:
    """``x2[:, width:width+Rp] = x2[:, :width] . operand^T`` (operand: [Rp, width] row view, rows past
    16*nct zero) -- the rank-r product of an augmented GEMM written into the operand's own spare
    columns.  The HIP skinny-GEMM kernel streams x2 once at HBM rate (csrc/kernels/swiglu_lora.hip
    ``tail_gemm``); elsewhere a GEMM into the strided tail."""
    xv = x2[:, :width] if x2.shape[1] != width else x2
    # up to 32 live columns the kernel streams at 6.3 TB/s vs hipBLASLt's 5.4 in isolation; at 48
    # (packed q|k|v forward, nct = 3) its L2 fragment traffic loses (tools/bench_rmsnorm.py).  End to
    # end the difference is within box noise (profiles/r1_tail_gemm_ab.log)
    if _HIP_TAIL and nct <= _HIP_TAIL_MAX_NCT and use_hip(x2) and ext().tail_gemm_ok(xv, Rp):
        ext().tail_gemm_(xv, operand, nct, Rp)
    else:
        _mm_into(x2, operand.t(), _tail(x2, width, Rp))


def _wide(t: torch.Tensor, width: int) -> torch.Tensor:
    return t.as_strided((t.shape[0], width), (t.stride(0), 1), t.storage_offset())


class AugWeight(_Refreshable):
    """``big [N+Rp, K+Rp]`` bf16 buffer whose ``[:N, :K]`` block is the frozen base weight."""

    TILE = 64

    def __init__(self, N: int, K: int, R: int, device=None, dtype=torch.bfloat16):
        self.N, self.K, self.R = N, K, R
        self.Rp = -(-R // self.TILE) * self.TILE
        self.big = torch.zeros(N + self.Rp, K + self.Rp, device=device, dtype=dtype)

    @property
    def W(self) -> torch.Tensor:
        return self.big[:self.N, :self.K]

    def owns(self, W: torch.Tensor) -> bool:
        return W.data_ptr() == self.big.data_ptr() and W.shape == (self.N, self.K) and W.stride(0) == self.K + self.Rp

    def _copy_jobs(self, A, B, scale) -> list:
        """big[:N, K:K+R] = B ; big[N:N+R, :K] = s A (pad rows / columns stay zero); bigT / bt follow.

        ``refresh`` runs them once per parameter update, not per call: forward and backward of every
        micro-batch between two optimizer steps see the same A/B (key = optimizer generation + the
        tensors' version counters and storage)."""
        N, K, R = self.N, self.K, self.R
        jobs = [(self.big[:N, K:K + R], B, 1.0), (self.big[N:N + R, :K], A, scale)]
        if self.bigT is not None:
            jobs.append((self.bigT[:, N:N + R], A.t(), scale))
        if self.bt is not None:
            jobs.append((self.bt[:R], B.t(), 1.0))
        return jobs

    # ---- producer-side tail products (csrc/kernels/swiglu_lora.hip): the kernel that produces this
    # projection's input (forward) or output gradient (backward) forms s x A^T / dy B itself.
    bt: torch.Tensor | None = None  # B^T [Rp, N] (rows past R zero), kept only when a producer asks

    @property
    def nct(self) -> int:
        """16-wide column tiles that hold the R live tail columns."""
        return -(-self.R // 16)

    def fwd_tail_operand(self, A: torch.Tensor, B: torch.Tensor, scale: float) -> torch.Tensor:
        """[Rp, K] row view of [s A ; 0] (refreshed)."""
        self.refresh(A, B, scale)
        return self.big[self.N:, :self.K]

    def bwd_tail_operand(self, A: torch.Tensor, B: torch.Tensor, scale: float) -> torch.Tensor:
        """[Rp, N] contiguous B^T (refreshed)."""
        if self.bt is None:
            self.bt = torch.zeros(self.Rp, self.N, device=self.big.device, dtype=self.big.dtype)
            self._key = None
        self.refresh(A, B, scale)
        return self.bt

    # ---- backward operand in the "TN" layout.  hipBLASLt runs dx = [dy | dyB] . [W ; sA] 14-16 %
    # faster when the right operand is stored K-contiguous (tools/bench_gemm_layouts.py), so a
    # transposed copy bigT [K, N+Rp] of the frozen weight is kept (HBM is plentiful: +2 B/param).
    # It is rebuilt lazily after invalidate() -- called wherever the base weight is rewritten
    # (init_weights, HF checkpoint load, LoRA merge/unmerge).
    bigT: torch.Tensor | None = None

    def invalidate(self):
        self.bigT = None
        self.bt = None
        self._key = None

    def bwd_operand(self) -> torch.Tensor:
        """[N+Rp, K] view of [W ; s A ; 0] with unit stride along N+Rp (column-major for the GEMM).
        Call after refresh(): the s A rows are copied from big."""
        N, K = self.N, self.K
        if self.bigT is None:
            self.bigT = torch.zeros(K, N + self.Rp, device=self.big.device, dtype=self.big.dtype)
            self.bigT[:, :N + self.R].copy_(self.big[:N + self.R, :K].t())
        return self.bigT.t()


def direct_grad_params(A, B, blocks):
    """(A, B) when both have a flat-buffer ``main_grad``, else None."""
    if (A is not None and getattr(A, "main_grad", None) is not None
            and getattr(B, "main_grad", None) is not None):
        return (A, B)
    return None


_HIP_WGRAD = True


def _accum_xty(out: torch.Tensor, X: torch.Tensor, Y: torch.Tensor, alpha: float, blocks=None):
    """out [M, R] += alpha * X^T Y for X [T, M], Y [T, R] with T = tokens: one streaming pass over X
    (csrc/kernels/lora_wgrad.hip: split-T MFMA + deterministic split reduction) where supported,
    else beta=1 GEMMs.  ``blocks`` (r0, r1, c0, c1): only those diagonal blocks of out are formed
    (block-diagonal B of a packed projection) -- one launch for all of them."""
    hip = _HIP_WGRAD and use_hip(X) and out.dtype == X.dtype
    if blocks is None:
        if hip and ext().lora_wgrad_ok(X, Y, Y.shape[1]):
            ext().lora_wgrad_(out, X, Y, Y.shape[1], float(alpha), 1.0)
        else:
            accum_mm(out, X.t(), Y, alpha)
        return
    R = blocks[0][3] - blocks[0][2]
    segs_ok = (len(blocks) <= 4 and blocks[0][0] == 0 and blocks[-1][1] == X.shape[1]
               and all(b[3] - b[2] == R and b[1] % 128 == 0 for b in blocks)
               and all(blocks[i][0] == blocks[i - 1][1] for i in range(1, len(blocks))))
    if hip and segs_ok and ext().lora_wgrad_ok(X, Y, R):
        ext().lora_wgrad_(out, X, Y, R, float(alpha), 1.0, [b[1] for b in blocks], [b[2] for b in blocks],
                          [b[2] for b in blocks])
    else:
        for r0, r1, c0, c1 in blocks:
            _accum_xty(out[r0:r1, c0:c1], X[:, r0:r1], Y[:, c0:c1], alpha)


def lora_weight_grads(direct, dy2, xa, xa_scaled, dyb, xin, s, blocks, need_a, need_b):
    """dB = dy^T (s x A^T), dA = s (dy B)^T x.  With ``direct`` = (A, B) homed in the flat grad buffer
    they are accumulated in place by beta=1 GEMMs (alpha carries the scale) and the data-parallel
    grad-ready hook fires; (None, None) is returned.  Otherwise fresh tensors are returned for
    autograd to accumulate."""
    dA = dB = None
    if need_b:
        if direct is not None:
            mg, alpha = direct[1].main_grad, 1.0 if xa_scaled else s
            # block-diagonal B of a packed projection: only the diagonal blocks have gradients
            _accum_xty(mg, dy2, xa, alpha, blocks)
            _grad_ready(direct[1])
        else:
            dB = torch.mm(dy2.t(), xa)
            if not xa_scaled:
                dB.mul_(s)
            dB = _mask_blocks(dB, blocks)
    if need_a:
        if direct is not None:
            _accum_xty(direct[0].main_grad.t(), xin, dyb, s)  # dA^T [K, R] += s x^T (dy B)
            _grad_ready(direct[0])
        else:
            dA = torch.mm(dyb.t(), xin).mul_(s)
    return dA, dB


class _LoRALinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, bias, A, B, scale, blocks, aug, p_drop=0.0, rope=None):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        mask = None
        if A is not None and p_drop > 0.0:
            # LoRA dropout (PEFT semantics: on the adapter input only); the two-GEMM path keeps the
            # base GEMM on the clean x.  The bool mask is saved; the dropped x is recomputed in backward.
            mask = torch.rand(x2.shape, device=x2.device, dtype=torch.float32) >= p_drop
            aug = None
        N, K = W.shape
        rope_of = rope
        # allocate the output in its final shape: the returned tensor must not be a view (RoPE
        # rotates it in place downstream)
        out = torch.empty(*shp[:-1], N, dtype=x.dtype, device=x.device)
        y = out.view(-1, N)
        xa = None
        use_aug = (aug is not None and A is not None and bias is None and aug.owns(W)
                   and _spare_cols(x2, K, aug.Rp))
        if use_aug:
            Rp = aug.Rp
            aug.refresh(A, B, scale)
            # [s x A^T | 0] straight into the spare columns of the producer's buffer (unless the
            # producer kernel already formed it: ops.activation.swiglu)
            if not take_prefilled("fwd", x2, aug):
                tail_product(x2, K, Rp, aug.big[N:, :K], aug.nct)
            xa = _tail(x2, K, aug.R)  # = s * x A^T
            torch.mm(_wide(x2, K + Rp), aug.big[:N].t(), out=y)  # hipBLASLt (K5 base GEMM: docs/kernels.md)
        else:
            if bias is None:
                torch.mm(x2, W.t(), out=y)
            else:
                torch.addmm(bias, x2, W.t(), out=y)
            if A is not None:
                xin = x2 if mask is None else x2 * mask / (1.0 - p_drop)
                xa = xin @ A.t()
                y.addmm_(xa, B.t(), alpha=scale)
        if use_aug:
            # the frozen W shares big's version counter, which the s*B / s*A refreshes bump: keep it
            # outside save_for_backward (it never changes while the graph lives)
            ctx.save_for_backward(x2, None, A, B, xa)
            ctx.W = W.detach()
        else:
            ctx.save_for_backward(x2, W, A, B, xa)
            ctx.W = None
        ctx.scale, ctx.blocks, ctx.shp, ctx.has_bias, ctx.aug = scale, blocks, shp, bias is not None, aug
        ctx.aug_fwd = use_aug  # saved xa is s * x A^T
        ctx.mask, ctx.p_drop = mask, p_drop
        ctx.rope = rope_of  # the rotation the backward undoes on dy
        if rope is not None:  # not fused into the GEMM: rotate the output in place (csrc/kernels/elementwise.hip)
            cos, sin, pos, seq_len, n_rot, hd = rope[:6]
            ext().rope_(y, cos, sin, pos, n_rot, hd, seq_len, False)
        # trainable A/B homed in a flat grad buffer (FlatAdamW sets .main_grad): their weight
        # gradients are accumulated in place by beta=1 GEMMs instead of returned (no temporaries, no
        # scale / accumulate kernels).  Block-masked packed pairs keep the returned-gradient path.
        ctx.lora_params = direct_grad_params(A, B, blocks)
        return out

    @staticmethod
    def backward(ctx, dy):
        join_wgrad_stream()  # the previous projection's side-stream dW (see _wgrad_on_side)
        if ctx.rope is not None and not (len(ctx.rope) > 6 and ctx.rope[6] is not None and ctx.rope[6].taken):
            # output was rope(x W^T ...): the gradient of the un-rotated product is the inverse rotation
            # (unless the consumer -- the flash backward -- already emitted it: ops.attention.RopeGrad)
            cos, sin, pos, seq_len, n_rot, hd = ctx.rope[:6]
            if dy.dim() != 2 or dy.stride(1) != 1 or dy.stride(0) % 8:
                dy = dy.reshape(-1, dy.shape[-1]).contiguous()
            ext().rope_(dy, cos, sin, pos, n_rot, hd, seq_len, True)
        x2, W, A, B, xa = ctx.saved_tensors
        if W is None:
            W = ctx.W
        s = ctx.scale
        aug = ctx.aug
        N = W.shape[0]
        dy2 = dy.reshape(-1, dy.shape[-1])
        need_x, need_w, need_b, need_a, need_bb = ctx.needs_input_grad[:5]
        dx = dW = db = dA = dB = None
        dyb = None
        xa_scaled = ctx.aug_fwd
        side_dw = False
        if need_w and _DW_STREAM and use_hip(x2) and not torch.cuda.is_current_stream_capturing():
            mg = getattr(W, "main_grad", None)
            if mg is not None:
                # issued before the input-gradient GEMM so that the two run concurrently
                _wgrad_on_side(mg, dy2, x2, _TN_DW, take_fresh(W, mg))
                side_dw = True
        if (need_x and aug is not None and A is not None and aug.owns(W) and _spare_cols(dy2, N, aug.Rp)):
            # dx = [dy | dy B | 0] . [W ; s A ; 0]: dy B lands in the spare columns of the producer's buffer
            Rp = aug.Rp
            aug.refresh(A, B, s)
            if not take_prefilled("bwd", dy2, aug):
                tail_product(dy2, N, Rp, aug.bwd_tail_operand(A, B, s), aug.nct)
            dyb = _tail(dy2, N, aug.R)
            rhs = aug.bwd_operand() if _TN_BWD else aug.big[:, :aug.K]
            dx = torch.empty(dy2.shape[0], aug.K, dtype=dy2.dtype, device=dy2.device)
            torch.mm(_wide(dy2, N + Rp), rhs, out=dx)
            dx = dx.view(ctx.shp)
        else:
            if A is not None and (need_x or need_a):
                dyb = dy2 @ B  # [T, R]
            if need_x:
                WT = transposed_weight(W)
                dx = dy2 @ W if WT is None else torch.mm(dy2, WT.t())
                if dyb is not None:
                    if ctx.mask is None:
                        dx.addmm_(dyb, A, alpha=s)
                    else:
                        dx.add_((dyb @ A) * ctx.mask, alpha=s / (1.0 - ctx.p_drop))
                dx = dx.view(ctx.shp)
        if need_w:
            mg = getattr(W, "main_grad", None)
            if mg is not None:
                if side_dw:
                    pass  # issued above, on the side stream
                elif _TN_DW and use_hip(x2):
                    # hipBLASLt runs dW += dy^T x 14-24 % faster with x handed over transposed (K-major
                    # reduction operand, tools/bench_dw_gemm.py); the transpose streams at HBM rate
                    wgrad_mm(mg, dy2.t(), transpose2d(x2).t(), beta=take_fresh(W, mg))
                else:
                    wgrad_mm(mg, dy2.t(), x2, beta=take_fresh(W, mg))
                _grad_ready(W)
            else:
                dW = dy2.t() @ x2
        if need_b and ctx.has_bias:
            db = dy2.sum(0)
        if A is not None and (need_a or need_bb):
            if need_a and dyb is None:
                dyb = dy2 @ B
            xin = x2 if ctx.mask is None else x2 * ctx.mask / (1.0 - ctx.p_drop)
            dA, dB = lora_weight_grads(ctx.lora_params, dy2, xa, xa_scaled, dyb, xin, s, ctx.blocks, need_a, need_bb)
        return dx, dW, db, dA, dB, None, None, None, None, None


def lora_linear(x: torch.Tensor, W: torch.Tensor, A: torch.Tensor | None = None, B: torch.Tensor | None = None,
                scale: float = 1.0, bias: torch.Tensor | None = None, blocks=None,
                aug: AugWeight | None = None, dropout: float = 0.0, rope: tuple | None = None) -> torch.Tensor:
    """``rope`` (GPU, bf16, 2-D x): ``(cos, sin, positions int32 | None, seq_len, n_rot_heads, head_dim
    [, RopeGrad])`` -- the output's first n_rot heads are rotated (RoPE, HF rotate_half) inside the op: in
    the GEMM epilogue when the hand-written kernel runs the projection, else in place right after it; the
    backward undoes the rotation on the incoming gradient, unless the optional ``ops.attention.RopeGrad``
    handoff was taken by the consumer (the flash backward then emits dq / dk already un-rotated)."""
    return _LoRALinearFn.apply(x, W, bias, A, B, scale, blocks, aug, float(dropout), rope)
