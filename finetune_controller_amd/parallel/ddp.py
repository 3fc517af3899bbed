"""Bucketed, backward-overlapped gradient all-reduce over the flat grad buffer (N1).

The optimizer (``train.optim.FlatAdamW``) lays every trainable parameter's gradient out in ONE
flat buffer in the order backward produces them.  This module cuts that buffer into contiguous
buckets of ``bucket_mb`` and launches an asynchronous SUM all-reduce of a bucket the moment the
last gradient inside it has been written -- while backward keeps computing earlier layers.  No
gradient is ever copied into or out of a staging buffer.

Readiness signals:
* parameters whose grads flow through autograd's ``AccumulateGrad`` (LoRA A/B, norms, embeddings)
  -> ``register_post_accumulate_grad_hook``;
* frozen-shape base weights in full fine-tuning, whose GEMM backward adds straight into
  ``main_grad`` -> the ``ops.linear`` grad-ready hook.

Parameters used more than once per step (tied embeddings) are deferred to ``finish()``.

ZeRO-1 (``train.optim.ShardedFlatAdamW``): the optimizer owns the bucket plan (every bucket padded
to a multiple of the world size) and each ready bucket is REDUCE-SCATTERED into the rank's owned
slice (``grad_shard``) instead of all-reduced -- half the bytes per rank on the wire during backward;
the updated parameters come back with an in-place all-gather after the optimizer step.

Transport: ``torch.distributed`` (ProcessGroupNCCL == RCCL over xGMI on MI355X; gloo on CPU), or the
native engine in ``parallel.comm`` (own RCCL communicator + dedicated high-priority HIP stream)
with ``engine="native"``.  Averaging is NOT done here: the optimizer folds 1/world into its
device-side grad scale, saving a full pass over the buffer.

Wire dtype (``wire_dtype``): with an fp32 gradient buffer (full FT with accumulation / data parallelism:
exact local accumulation) the reduction may still travel as bf16 -- each ready bucket is cast into a bf16
staging buffer, reduced (reduce-scattered under ZeRO-1) in bf16 and cast back into the fp32 owned slice
when it is waited for.  Half the bytes on the wire (Llama-3-8B ZeRO-1 on 8 ranks: the 28 GB fp32
reduce-scatter becomes 14 GB per rank per step) for one bf16 rounding of each rank's partial sum plus the
ring's bf16 adds (``tests/test_distributed.py`` bounds the drift against an fp64 reference).

Bucket sizing for MI355X: each GPU has 7 xGMI links of ≈153 GB/s; a ring
all-reduce is per-link bound, so buckets must be large enough for RCCL to spread over several
channels (default 64 MB) but small enough that the last bucket -- which cannot overlap -- stays
short.  LoRA grads (27-84 MB) fit 1-2 buckets; full FT (16 GB bf16) ~250 buckets.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import linear as _linear


class GradBucketer:
    def __init__(self, optimizer, bucket_mb: float = 64.0, group=None, engine: str = "torch",
                 multi_use_params=(), wire_dtype: torch.dtype | None = None):
        self.opt = optimizer
        self.group = group
        self.engine = engine
        # the reduction's dtype on the wire: None / the buffer's dtype = reduce in place
        gd = optimizer.grad_flat.dtype
        self.wire_dtype = None if wire_dtype in (None, gd) else wire_dtype
        if self.wire_dtype is not None and (gd != torch.float32 or self.wire_dtype != torch.bfloat16):
            raise ValueError(f"gradient wire {wire_dtype} over a {gd} buffer: only bf16 over fp32 is supported")
        self.enabled = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        self.world = dist.get_world_size(group) if self.enabled else 1
        self.sharded = hasattr(optimizer, "grad_shard")  # ZeRO-1 (train.optim.ShardedFlatAdamW)
        multi = {id(p) for p in multi_use_params}
        self.deferred = []
        self.deferred_buckets: set[int] = set()
        self.buckets: list[tuple[int, int]] = []  # (start, end) element ranges of grad_flat
        self.param_bucket: dict[int, int] = {}
        members: list[list[int]] = [[]]
        if self.sharded:
            # the optimizer owns the bucket plan (buckets padded to a multiple of world, one owned
            # slice per rank); a bucket holding a multi-use parameter waits for finish()
            self.buckets = list(optimizer.buckets)
            members = []
            for b, ps in enumerate(optimizer.bucket_params):
                members.append([id(p) for p in ps if id(p) not in multi])
                if any(id(p) in multi for p in ps):
                    self.deferred_buckets.add(b)
        else:
            esize = optimizer.grad_flat.element_size()
            cap = max(1, int(bucket_mb * 1024 * 1024 / esize))
            start = 0
            cur_end = 0
            for p, (o, n) in zip(optimizer.params, optimizer.offsets):
                if id(p) in multi:
                    self.deferred.append((o, n))
                    continue
                if cur_end - start >= cap and members[-1]:
                    self.buckets.append((start, cur_end))
                    members.append([])
                    start = cur_end
                members[-1].append(id(p))
                cur_end = o + n
            if members[-1]:
                self.buckets.append((start, cur_end))
        self.members = members
        for b, ids in enumerate(members):
            if b in self.deferred_buckets:
                continue
            for pid in ids:
                self.param_bucket[pid] = b
        self._native = None
        if self.enabled and engine == "native":
            from .comm import NativeAllReduce

            self._native = NativeAllReduce(group)
        self.armed = True  # False on non-final micro-batches of gradient accumulation
        self._hooks = []
        if self.enabled:
            for p in optimizer.params:
                if id(p) in self.param_bucket:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
            _linear.set_grad_ready_hook(self._on_grad)
        self.reset()

    def reset(self):
        self.remaining = [len(m) for m in self.members]
        self.seen: set[int] = set()
        self.works = []
        self.unstage = []  # bf16 wire: (reduced bf16 buffer, fp32 destination) to cast back after the waits
        self.launched = [False] * len(self.buckets)

    def _on_grad(self, p):
        if not self.armed:
            return
        pid = id(p)
        b = self.param_bucket.get(pid)
        if b is None or pid in self.seen:
            return
        self.seen.add(pid)
        self.remaining[b] -= 1
        if self.remaining[b] == 0:
            self._launch(b)

    def _launch(self, b: int):
        if self.launched[b]:
            return
        self.launched[b] = True
        side = _linear.wgrad_launch_stream()
        if side is not None:  # weight gradients are being written on the side stream: enqueue behind them
            with torch.cuda.stream(side):
                return self._launch_now(b)
        return self._launch_now(b)

    def _launch_now(self, b: int):
        s, e = self.buckets[b]
        view = self.opt.grad_flat[s:e]
        if self.sharded:
            out = self.opt.shard_view(b, self.opt.grad_shard)
            if self.wire_dtype is not None:  # fp32 buffer, bf16 on the wire (staging freed after the wait)
                view = view.to(self.wire_dtype)
                dst, out = out, torch.empty(out.numel(), dtype=self.wire_dtype, device=out.device)
                self.unstage.append((out, dst, view))
            if self._native is not None:
                self.works.append(self._native.reduce_scatter_async(out, view))
            else:
                self.works.append(dist.reduce_scatter_tensor(out, view, group=self.group, async_op=True))
            return
        self._all_reduce(view)

    def _all_reduce(self, view):
        if self.wire_dtype is not None:
            dst, view = view, view.to(self.wire_dtype)
            self.unstage.append((view, dst, None))
        if self._native is not None:
            self.works.append(self._native.all_reduce_async(view))
        else:
            self.works.append(dist.all_reduce(view, group=self.group, async_op=True))

    def finish(self):
        """Launch anything not yet launched (unused params, deferred tied weights) and wait."""
        _linear.gradients_final()  # a bucket still unlaunched may hold a skipped weight this step never wrote
        if not self.enabled:
            if self.sharded:  # world 1: the owned slice is the whole bucket
                for b, (s, e) in enumerate(self.buckets):
                    self.opt.shard_view(b, self.opt.grad_shard).copy_(self.opt.grad_flat[s:e])
            return
        for b in range(len(self.buckets)):
            if not self.launched[b]:
                self._launch(b)
        for o, n in self.deferred:
            self._all_reduce(self.opt.grad_flat[o:o + n])
        for w in self.works:
            w.wait()
        for red, dst, inp in self.unstage:  # bf16 wire: the reduced sums back into the fp32 buffer
            dst.copy_(red)
            if red.is_cuda:
                # both staging blocks were allocated on the launch (maybe side) stream and used by the
                # collective on the comm stream (the native engine records nothing on its own stream).
                # The current stream has waited for that collective, so recording them here keeps each
                # block out of the side stream's pool until the collective's reads and this copy ran.
                cur = torch.cuda.current_stream(red.device)
                red.record_stream(cur)
                if inp is not None:
                    inp.record_stream(cur)
        if self._native is not None:
            self._native.reset()
        self.reset()

    def n_collectives(self) -> int:
        """Gradient collectives per optimizer step (buckets + deferred multi-use parameters)."""
        return len(self.buckets) + len(self.deferred) if self.enabled else 0

    def wire_bytes_per_step(self) -> int:
        """Bytes each rank sends per optimizer step for the gradient reduction (and, under ZeRO-1, the
        parameter all-gather), ring-equivalent: an all-reduce of S bytes moves 2 (n-1)/n S, a
        reduce-scatter or all-gather (n-1)/n S (nccl-tests bus-bandwidth convention)."""
        if not self.enabled:
            return 0
        n = self.world
        g = (torch.empty((), dtype=self.wire_dtype).element_size() if self.wire_dtype is not None
             else self.opt.grad_flat.element_size())
        if self.sharded:
            red = sum(e - s for s, e in self.buckets) * g * (n - 1) / n
            gather = sum(e - s for s, e in self.buckets) * self.opt.param_flat.element_size() * (n - 1) / n
        else:
            red = sum(e - s for s, e in self.buckets) * g * 2 * (n - 1) / n
            gather = 0
        red += sum(k for _, k in self.deferred) * g * 2 * (n - 1) / n
        return int(red + gather)

    def close(self):
        for h in self._hooks:
            h.remove()
        _linear.set_grad_ready_hook(None)
