"""Ulysses sequence parallelism (SP) for the decoder's attention.

Long contexts beyond one GPU's activation budget: the P ranks of a sequence-parallel group hold the
SAME sequences, each rank a contiguous 1/P of every sequence's tokens.  Everything per token
(embedding, norms, the LoRA / full projections, SwiGLU, the chunked CE) runs on the local tokens
unchanged; only attention needs the whole sequence, and it gets it by switching the sharding from
tokens to heads with one all-to-all before and one after it:

    qkv [B*S/P, (H + 2KV) D]  --all-to-all-->  [B*S, (H/P + 2 KV/P) D]   (all tokens, this rank's heads)
    flash attention (causal over the FULL sequence, H/P query heads on KV/P kv heads: GQA groups
    stay whole because rank r takes q heads [r H/P, (r+1) H/P) and kv heads [r KV/P, (r+1) KV/P))
    out [B*S, H/P D]          --all-to-all-->  [B*S/P, H D]              (this rank's tokens, all heads)

Why Ulysses and not a ring: on the MI355X node every GPU pair has its own xGMI link,
so an all-to-all drives all 7 links of every GPU at once, while ring attention's neighbour exchange
uses one or two; the all-to-all volume per layer is 4 x the layer's activations / P, independent of
the sequence length's square.  Gradients: every rank holds full weight replicas and computes partial
weight gradients over its tokens, so the data-parallel all-reduce (``parallel.ddp``, averaging over
the whole world) is also the sequence-parallel reduction -- the global mean loss's gradient when the
ranks see equal token counts.

No reference counterpart (the reference has no training code); the transport is
``torch.distributed.all_to_all_single`` (RCCL over xGMI on the GPU, gloo on the CPU tests).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class SeqGroup:
    group: object  # torch.distributed ProcessGroup of the P ranks sharing the sequences
    size: int      # P
    rank: int      # this rank's index in the group = which 1/P of every sequence it holds

    def positions(self, B: int, S_local: int, device) -> torch.Tensor:
        """Absolute positions of the local tokens, row after row: RoPE needs them global."""
        p = torch.arange(S_local, device=device, dtype=torch.int32) + self.rank * S_local
        return p.repeat(B)


def make_seq_groups(sp: int, world: int, rank: int) -> tuple[SeqGroup | None, int, int]:
    """Consecutive ranks form the sequence-parallel groups ([0, sp), [sp, 2 sp), ...).  Returns (this
    rank's SeqGroup or None for sp == 1, data-parallel index, data-parallel size).  Every rank must call
    this (``new_group`` is collective)."""
    if sp <= 1:
        return None, rank, world
    if world % sp:
        raise ValueError(f"sequence parallel degree {sp} does not divide the world size {world}")
    mine = None
    for g in range(world // sp):
        ranks = list(range(g * sp, (g + 1) * sp))
        pg = dist.new_group(ranks)
        if rank in ranks:
            mine = SeqGroup(pg, sp, rank - g * sp)
    return mine, rank // sp, world // sp


def _a2a(send: torch.Tensor, group) -> torch.Tensor:
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    return recv


def _tokens_to_heads(qkv: torch.Tensor, B: int, Sl: int, H: int, KV: int, D: int, sp: SeqGroup) -> torch.Tensor:
    """[B*Sl, (H+2KV) D] (row view; extra columns ignored) -> [B*P*Sl, (H/P + 2 KV/P) D] contiguous.

    The send buffer is filled by three strided copies straight from the projection output (one pass
    over qkv, no concatenation temporary); with B == 1 the received [P(src), Sl, C, D] buffer already is
    the token-major [P*Sl, C*D] row layout the flash kernels read, so it is returned without a copy."""
    P = sp.size
    Hp, KVp = H // P, KV // P
    C = Hp + 2 * KVp
    x = qkv[:, :(H + 2 * KV) * D]
    send = torch.empty(P, B, Sl, C, D, dtype=qkv.dtype, device=qkv.device)
    sv = send.permute(1, 2, 0, 3, 4)  # [B, Sl, P, C, D] view of the send buffer
    sv[:, :, :, :Hp].copy_(x[:, :H * D].reshape(B, Sl, P, Hp, D))
    sv[:, :, :, Hp:Hp + KVp].copy_(x[:, H * D:(H + KV) * D].reshape(B, Sl, P, KVp, D))
    sv[:, :, :, Hp + KVp:].copy_(x[:, (H + KV) * D:].reshape(B, Sl, P, KVp, D))
    recv = _a2a(send, sp.group)                                                 # [P(src), B, Sl, C, D]
    if B == 1:
        return recv.view(P * Sl, C * D)
    return recv.permute(1, 0, 2, 3, 4).reshape(B * P * Sl, C * D)


def _heads_to_tokens_qkv(g: torch.Tensor, B: int, Sl: int, H: int, KV: int, D: int, sp: SeqGroup) -> torch.Tensor:
    """Inverse of ``_tokens_to_heads``: [B*P*Sl, (H/P + 2 KV/P) D] -> [B*Sl, (H+2KV) D]."""
    P = sp.size
    Hp, KVp = H // P, KV // P
    C = Hp + 2 * KVp
    send = g.reshape(B, P, Sl, C, D).permute(1, 0, 2, 3, 4).contiguous()  # [P(dst tokens), B, Sl, C, D]
    recv = _a2a(send, sp.group)                                          # [P(src heads), B, Sl, C, D]
    r = recv.permute(1, 2, 0, 3, 4)                                      # [B, Sl, P, C, D]
    q = r[..., :Hp, :].reshape(B * Sl, H * D)
    k = r[..., Hp:Hp + KVp, :].reshape(B * Sl, KV * D)
    v = r[..., Hp + KVp:, :].reshape(B * Sl, KV * D)
    return torch.cat([q, k, v], dim=1)


def _heads_to_tokens(a: torch.Tensor, B: int, Sl: int, nh: int, D: int, sp: SeqGroup) -> torch.Tensor:
    """Attention output [B*P*Sl, nh/P D] -> [B*Sl, nh D] (this rank's tokens, every head)."""
    P = sp.size
    # B == 1: the output rows already are [P(dst tokens), Sl, ...] -- sent as they are
    send = a.reshape(B, P, Sl, nh // P, D).permute(1, 0, 2, 3, 4)
    send = send.contiguous() if B > 1 else send.reshape(P, 1, Sl, nh // P, D)
    recv = _a2a(send, sp.group)                                          # [P(src heads), B, Sl, nh/P, D]
    return recv.permute(1, 2, 0, 3, 4).reshape(B * Sl, nh * D)


def _tokens_to_heads_out(g: torch.Tensor, B: int, Sl: int, nh: int, D: int, sp: SeqGroup) -> torch.Tensor:
    """Inverse of ``_heads_to_tokens``: [B*Sl, nh D] -> [B*P*Sl, nh/P D]."""
    P = sp.size
    send = g.reshape(B, Sl, P, nh // P, D).permute(2, 0, 1, 3, 4).contiguous()
    recv = _a2a(send, sp.group)
    return recv.permute(1, 0, 2, 3, 4).reshape(B * P * Sl, (nh // P) * D)


class _QKVToHeads(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, B, Sl, H, KV, D, sp):
        ctx.args = (B, Sl, H, KV, D, sp)
        ctx.width = qkv.shape[1]
        return _tokens_to_heads(qkv, B, Sl, H, KV, D, sp)

    @staticmethod
    def backward(ctx, g):
        B, Sl, H, KV, D, sp = ctx.args
        dx = _heads_to_tokens_qkv(g.contiguous(), B, Sl, H, KV, D, sp)
        if ctx.width != dx.shape[1]:  # qkv was a column view of a wider (LoRA-padded) buffer
            dx = torch.nn.functional.pad(dx, (0, ctx.width - dx.shape[1]))
        return dx, None, None, None, None, None, None


class _OutToTokens(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, B, Sl, nh, D, sp):
        ctx.args = (B, Sl, nh, D, sp)
        return _heads_to_tokens(a.contiguous(), B, Sl, nh, D, sp)

    @staticmethod
    def backward(ctx, g):
        B, Sl, nh, D, sp = ctx.args
        return _tokens_to_heads_out(g.contiguous(), B, Sl, nh, D, sp), None, None, None, None, None


def sp_attention(qkv: torch.Tensor, B: int, S_local: int, H: int, KV: int, D: int, window: int,
                 sp: SeqGroup) -> torch.Tensor:
    """Causal GQA attention over the full sequence of a sequence-parallel group; ``qkv`` holds this
    rank's ``S_local`` tokens of each of the B sequences (RoPE applied with global positions).  Returns
    this rank's tokens' attention output [B*S_local, H*D]."""
    from ..ops.attention import attention_packed

    P = sp.size
    if H % P or KV % P:
        raise ValueError(f"sequence parallel degree {P} must divide the query ({H}) and kv ({KV}) head counts")
    full = _QKVToHeads.apply(qkv, B, S_local, H, KV, D, sp)
    a = attention_packed(full, B, P * S_local, H // P, KV // P, D, True, window)
    return _OutToTokens.apply(a, B, S_local, H, D, sp)


def shard_batch(x: torch.Tensor, y: torch.Tensor, sp: SeqGroup) -> tuple[torch.Tensor, torch.Tensor]:
    """This rank's contiguous 1/P of every row of a [B, S] batch (inputs and labels alike: the label of
    a chunk's last token is the next chunk's first input, already in ``y``)."""
    S = x.shape[-1]
    if S % sp.size:
        raise ValueError(f"seq_len {S} is not divisible by the sequence parallel degree {sp.size}")
    Sl = S // sp.size
    lo = sp.rank * Sl
    y = y.reshape(x.shape)
    return x[:, lo:lo + Sl].contiguous(), y[:, lo:lo + Sl].contiguous()


class SeqShard:
    """Data wrapper: every rank of an SP group draws the same [B, S] batch and keeps its contiguous
    1/P of each row (``shard_batch``).

    Loss normaliser: a masked batch (document boundaries, completion-only prompts) leaves the P shards
    different valid-token counts, so each rank divides its local loss sum by the WHOLE batch's count
    over P (``last_n_valid``, counted host-side by the source on the full batch): the mean over the
    group's ranks is then the batch's mean loss exactly, and so is the all-reduced gradient."""

    def __init__(self, inner, sp: SeqGroup):
        self.inner, self.sp = inner, sp

    @property
    def last_n_valid(self):
        n = getattr(self.inner, "last_n_valid", None)
        return None if n is None else n / self.sp.size

    def __iter__(self):
        return self

    def __next__(self):
        return shard_batch(*next(self.inner), self.sp)

    def __getattr__(self, name):  # state(), load_state(), steps_per_epoch, ... of the wrapped source
        if name in ("inner", "sp"):
            raise AttributeError(name)
        return getattr(self.inner, name)
