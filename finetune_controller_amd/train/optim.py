"""Flat-buffer mixed-precision AdamW (K7 driver) and LR schedules.

All trainable parameters are re-homed into ONE flat buffer (``param_flat``, the model dtype) and
their gradients into ONE flat grad buffer (``grad_flat``); each ``p.data`` / ``p.grad`` /
``p.main_grad`` becomes a view.  Consequences:

* autograd accumulates straight into the flat grad buffer (``AccumulateGrad`` adds in place into an
  existing ``.grad``), and the custom GEMM backward of frozen-shape weights adds into
  ``main_grad`` with a beta=1 GEMM;
* the data-parallel all-reduce works on contiguous bucket slices of that buffer with no packing
  copies (``parallel.ddp``);
* the optimizer is one HIP launch for the global grad norm and one for AdamW over the whole
  buffer, with the clip coefficient and the 1/world averaging read from device memory -- no host
  synchronisation inside ``step()``.

Gradient precision (``grad_dtype``): by default the grad buffer has the model dtype.  With
``grad_dtype=torch.float32`` (full fine-tuning with gradient accumulation or data parallelism) the
buffer is fp32: the GEMM weight gradients accumulate into it with bf16 operands and an fp32 C
(``ops.linear.accum_mm``), gradients that autograd produces in the model dtype (norm weights,
embeddings) are folded in by a post-accumulate hook, and the data-parallel reduction sums fp32 --
no mantissa is lost across micro-batches or ranks.

Checkpoint format: ``state_dict`` holds the state per parameter with no padding ("compact"), so a
resume works across world sizes and with ZeRO-1 switched on or off (the flat layout pads buckets
to a multiple of the world size).

Layout: parameters are placed in REVERSE registration order (last layer first), i.e. in the order
backward produces their gradients, so the first DDP buckets become ready first.
"""
from __future__ import annotations

import math

import torch

from ..ops._backend import ext, use_hip
from ..ops import linear as _linear
from ..ops.linear import bump_param_generation

ALIGN = 64  # elements: keeps every view 128-byte aligned for 16-byte vector access


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class FlatAdamW:
    def __init__(self, params, lr: float = 2e-4, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 max_grad_norm: float = 1.0, grad_scale: float = 1.0, bucket_elems: int = 0, pad_multiple: int = 1,
                 grad_dtype: torch.dtype | None = None):
        seen, plist = set(), []
        for p in params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                plist.append(p)
        if not plist:
            raise ValueError("FlatAdamW: no trainable parameters")
        dtypes = {p.dtype for p in plist}
        if len(dtypes) != 1:
            raise ValueError(f"FlatAdamW: trainable params must share one dtype, got {dtypes}")
        self.dtype = plist[0].dtype
        self.device = plist[0].device
        _linear.reset_grad_owned()  # the gradients are re-homed below: nothing may skip zeroing yet
        self.params = list(reversed(plist))
        self.offsets: list[tuple[int, int]] = []
        # bucket plan (ZeRO-1 sharding): contiguous [start, end) ranges closed once they reach
        # bucket_elems, each padded to a multiple of pad_multiple elements so it splits evenly over ranks
        self.buckets: list[tuple[int, int]] = []
        self.bucket_params: list[list] = []
        self.bucket_elems = bucket_elems
        off = start = 0
        members: list = []
        quantum = ALIGN * max(1, pad_multiple)
        for p in self.params:
            self.offsets.append((off, p.numel()))
            off += _align(p.numel())
            members.append(p)
            if bucket_elems and off - start >= bucket_elems:
                off = -(-off // quantum) * quantum
                self.buckets.append((start, off))
                self.bucket_params.append(members)
                start, members = off, []
        if bucket_elems and members:
            off = -(-off // quantum) * quantum
            self.buckets.append((start, off))
            self.bucket_params.append(members)
        self.numel = off
        self.param_flat = torch.zeros(off, dtype=self.dtype, device=self.device)
        self.grad_dtype = grad_dtype or self.dtype
        self.grad_flat = torch.zeros(off, dtype=self.grad_dtype, device=self.device)
        self._fold_hooks = []
        with torch.no_grad():
            for p, (o, n) in zip(self.params, self.offsets):
                self.param_flat[o:o + n].copy_(p.detach().reshape(-1))
                p.data = self.param_flat[o:o + n].view_as(p)
                g = self.grad_flat[o:o + n].view_as(p)
                p.main_grad = g
                if self.grad_dtype == self.dtype:
                    p.grad = g  # autograd accumulates in place into the flat buffer
                else:
                    # autograd's gradient has the parameter's dtype: fold it into the wider buffer and
                    # drop it (registered before any data-parallel hook, so it runs first)
                    p.grad = None
                    self._fold_hooks.append(p.register_post_accumulate_grad_hook(_fold_grad))
        self._init_state()
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.grad_scale = grad_scale  # e.g. 1/world_size when grads are summed by all-reduce
        self.step_count = 0
        self.last_grad_norm: torch.Tensor | None = None
        self._hp_table: torch.Tensor | None = None  # device schedule (graph-captured steps)
        self._hp_idx: torch.Tensor | None = None
        self._stages: list[tuple[int, int]] | None = None  # overlapped update: flat ranges in forward order
        self._side: torch.cuda.Stream | None = None
        self._events: list | None = None  # per stage, recorded on the side stream by the last step

    def use_device_schedule(self, lrs: list[float]):
        """Read lr and the bias corrections from a device table, one row per coming step, indexed by a
        device counter the step itself advances: a step captured in a hipGraph then replays with the
        schedule instead of the capture-time constants.  Row i: [lrs[i], 1 - b1^t, 1 - b2^t] with
        t = step_count + 1 + i."""
        b1, b2 = self.betas
        rows = [[lr, 1.0 - b1 ** (self.step_count + 1 + i), 1.0 - b2 ** (self.step_count + 1 + i)]
                for i, lr in enumerate(lrs)]
        self._hp_table = torch.tensor(rows, dtype=torch.float32, device=self.device)
        self._hp_idx = torch.zeros(1, dtype=torch.long, device=self.device)

    def _init_state(self):
        self.master = self.param_flat.float() if self.dtype != torch.float32 else self.param_flat
        self.exp_avg = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.exp_avg_sq = torch.zeros(self.numel, dtype=torch.float32, device=self.device)

    @torch.no_grad()
    def sync_master(self):
        """Re-derive the fp32 master copy from ``param_flat`` (after a broadcast / external load)."""
        if self.master is not self.param_flat:
            self.master.copy_(self.param_flat)

    def num_params(self) -> int:
        return sum(n for _, n in self.offsets)

    # ---- update overlapped with the next forward (full fine-tuning)
    def enable_overlap(self, stages: list[list[torch.Tensor]]) -> bool:
        """Run the AdamW update stage by stage on a side stream so that the next step's forward can start
        on stage 0 (embeddings, then layer 0, ...) while later stages are still being updated; the model
        calls ``wait_stage(i)`` before it reads stage i's parameters.  ``stages``: the trainable
        parameters grouped in forward order; every parameter in exactly one stage, each stage a
        contiguous range of the flat layout.  The AdamW kernel is HBM-bound (28 B per parameter: 39 ms
        for Llama-3-8B) and the forward GEMMs are matrix-bound, so the two share the chip.  Each stage's
        gradient slice is zeroed on the side stream right after its update (the next ``zero_grad`` has
        nothing left to do: gradients are next written by the backward, after the forward has waited
        for every stage).  Returns False (nothing changed) when the layout does not allow it."""
        if not (use_hip(self.grad_flat) and self.dtype in (torch.bfloat16, torch.float32)):
            return False
        where = {id(p): (o, _align(n)) for p, (o, n) in zip(self.params, self.offsets)}
        ranges = []
        seen = 0
        for group in stages:
            spans = [where[id(p)] for p in group if id(p) in where]
            if not spans:
                continue
            lo, hi = min(o for o, _ in spans), max(o + n for o, n in spans)
            if sum(n for _, n in spans) != hi - lo:
                return False  # not contiguous in the flat layout
            ranges.append((lo, hi))
            seen += len(spans)
        if seen != len(self.params):
            return False
        self._stages = ranges
        self._side = torch.cuda.Stream(device=self.device)
        return True

    def wait_stage(self, i: int):
        """Make the current stream wait for the last update of stage i (no-op when none is pending)."""
        if self._events is not None and i < len(self._events):
            torch.cuda.current_stream(self.device).wait_event(self._events[i])

    def join(self):
        """Every pending stage update is ordered before the current stream's next work."""
        if self._events is not None:
            torch.cuda.current_stream(self.device).wait_event(self._events[-1])

    def zero_grad(self):
        if self._events is None:
            mine = [i for i, p in enumerate(self.params) if _linear.is_grad_owned(p)] if _linear._FIRST_WRITE else []
            if mine and not (self.grad_flat.is_cuda and torch.cuda.is_current_stream_capturing()):
                # projection weights: their first GEMM of the step overwrites (ops.linear take_fresh)
                key = tuple(mine)
                if getattr(self, "_zero_key", None) != key:
                    skip = set(mine)
                    runs, lo, hi = [], None, None
                    for i, (o, n) in enumerate(self.offsets):
                        end = self.offsets[i + 1][0] if i + 1 < len(self.offsets) else self.numel
                        if i in skip:
                            continue
                        if lo is not None and o == hi:
                            hi = end
                        else:
                            if lo is not None:
                                runs.append((lo, hi))
                            lo, hi = o, end
                    if lo is not None:
                        runs.append((lo, hi))
                    self._zero_key, self._zero_runs = key, [self.grad_flat[lo:hi] for lo, hi in runs]
                torch._foreach_zero_(self._zero_runs)  # one multi-tensor launch for the ~2 runs per layer
                _linear.mark_fresh(id(self.params[i]) for i in mine)
            else:
                self.grad_flat.zero_()
        if self._fold_hooks:
            for p in self.params:
                p.grad = None

    # ---- layout-independent (compact) views of flat-layout tensors
    def compact(self, flat: torch.Tensor, dtype: torch.dtype | None = None) -> torch.Tensor:
        """CPU copy of the live elements of a full-layout tensor, parameter after parameter."""
        out = torch.empty(self.num_params(), dtype=dtype or flat.dtype)
        i = 0
        for o, n in self.offsets:
            out[i:i + n].copy_(flat[o:o + n])
            i += n
        return out

    def expand_(self, compact: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        """Scatter a compact tensor into the full layout ``out`` (padding untouched)."""
        if compact.numel() != self.num_params():
            raise ValueError(f"checkpoint holds {compact.numel()} elements, this parameter set has {self.num_params()}")
        i = 0
        for o, n in self.offsets:
            out[o:o + n].copy_(compact[i:i + n])
            i += n
        return out

    def layout(self) -> list[int]:
        return [n for _, n in self.offsets]

    def export_params(self) -> torch.Tensor:
        return self.compact(self.param_flat)

    @torch.no_grad()
    def import_params(self, compact: torch.Tensor):
        self.expand_(compact.to(self.param_flat.dtype), self.param_flat)

    @torch.no_grad()
    def step(self, lr: float | None = None):
        _linear.gradients_final()  # side-stream dW joined, never-written skipped weights zeroed
        lr = self.lr if lr is None else lr
        self.step_count += 1
        bump_param_generation()  # the update below rewrites param_flat in place
        b1, b2 = self.betas
        if use_hip(self.grad_flat) and self.dtype in (torch.bfloat16, torch.float32):
            stats = ext().grad_sumsq(self.grad_flat, self.max_grad_norm, self.grad_scale)
            self.last_grad_norm = stats[0:1]
            param = self.param_flat if self.dtype == torch.bfloat16 else None
            hp = None
            if self._hp_table is not None:
                hp = self._hp_table.index_select(0, self._hp_idx.clamp(max=self._hp_table.shape[0] - 1)).reshape(3)
                self._hp_idx += 1
            if self._stages is None:
                ext().adamw_(param, self.master, self.exp_avg, self.exp_avg_sq, self.grad_flat, lr, b1, b2, self.eps,
                             self.wd, self.step_count, stats[1:2], hp)
                return
            main = torch.cuda.current_stream(self.device)
            side = self._side
            side.wait_stream(main)  # grads final, norm / clip coefficient computed
            stats.record_stream(side)
            if hp is not None:
                hp.record_stream(side)
            events = []
            with torch.cuda.stream(side):
                for lo, hi in self._stages:
                    ext().adamw_(param[lo:hi] if param is not None else None, self.master[lo:hi], self.exp_avg[lo:hi],
                                 self.exp_avg_sq[lo:hi], self.grad_flat[lo:hi], lr, b1, b2, self.eps, self.wd,
                                 self.step_count, stats[1:2], hp)
                    self.grad_flat[lo:hi].zero_()
                    ev = torch.cuda.Event()
                    ev.record(side)
                    events.append(ev)
            self._events = events
            return
        g = self.grad_flat.float() * self.grad_scale
        norm = g.norm()
        self.last_grad_norm = norm.pow(2).reshape(1)
        if self.max_grad_norm and self.max_grad_norm > 0:
            g = g * torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0)
        bc1, bc2 = 1 - b1 ** self.step_count, 1 - b2 ** self.step_count
        self.exp_avg.mul_(b1).add_(g, alpha=1 - b1)
        self.exp_avg_sq.mul_(b2).addcmul_(g, g, value=1 - b2)
        self.master.mul_(1 - lr * self.wd)
        self.master.addcdiv_(self.exp_avg / bc1, (self.exp_avg_sq / bc2).sqrt_().add_(self.eps), value=-lr)
        if self.master is not self.param_flat:
            self.param_flat.copy_(self.master)

    def grad_norm(self) -> float:
        if self.last_grad_norm is None:
            return 0.0
        return float(self.last_grad_norm.float().sqrt().item()) * (self.grad_scale if use_hip(self.grad_flat) else 1.0)

    def state_dict(self) -> dict:
        """Compact (unpadded, per-parameter) CPU state: loadable at any world size, ZeRO on or off."""
        return {"format": "compact", "layout": self.layout(), "master": self.compact(self.master, torch.float32),
                "exp_avg": self.compact(self.exp_avg), "exp_avg_sq": self.compact(self.exp_avg_sq),
                "step": self.step_count, "lr": self.lr}

    def _check_layout(self, sd: dict):
        if sd.get("format") != "compact":
            raise ValueError("optimizer checkpoint predates the compact format (resume it with the world size and "
                             "ZeRO setting that wrote it)")
        if list(sd["layout"]) != self.layout():
            raise ValueError("optimizer checkpoint does not match this model's trainable parameters "
                             f"({len(sd['layout'])} vs {len(self.offsets)} tensors)")

    @torch.no_grad()
    def load_state_dict(self, sd: dict):
        self._check_layout(sd)
        self.expand_(sd["master"], self.master)
        self.expand_(sd["exp_avg"], self.exp_avg)
        self.expand_(sd["exp_avg_sq"], self.exp_avg_sq)
        self.step_count = int(sd["step"])
        bump_param_generation()
        if self.master is not self.param_flat:
            self.param_flat.copy_(self.master)


class ShardedFlatAdamW(FlatAdamW):
    """ZeRO-1: the fp32 master weights and both AdamW moments are partitioned over the data-parallel
    ranks (1/world of the optimizer state per GPU: 96 GB -> 12 GB for Llama-3-8B full fine-tuning on
    8 x MI355X).

    The flat layout is cut into buckets padded to a multiple of ``world`` (``bucket_elems``); rank r
    owns slice r of every bucket.  ``parallel.ddp.GradBucketer`` reduce-scatters each bucket as soon
    as backward has produced it (``grad_shard`` receives the summed slice -- same bytes on the wire as
    half an all-reduce), ``step()`` updates the owned slices with the same HIP AdamW kernel (one launch
    per bucket, writing bf16 straight into ``param_flat``) after an all-reduced global grad norm, and
    the updated slices are all-gathered in place into every rank's ``param_flat``.

    Checkpoints (``state_dict``) hold the gathered state in the compact per-parameter format, so a
    run can resume on any world size or without ZeRO; ``state_dict`` is a collective call."""

    def __init__(self, params, world: int, rank: int, group=None, bucket_elems: int = 16 << 20, **kw):
        self.world, self.rank, self.group = world, rank, group
        super().__init__(params, bucket_elems=bucket_elems, pad_multiple=world, **kw)
        # parameter all-gather: one async collective per bucket, issued right after that bucket's AdamW in
        # the order the next forward reads the buckets; without gates (enable_gather_overlap) step() waits
        # for all of them itself
        self._pending: dict = {}  # bucket -> all-gather work not waited for yet
        self._stage_buckets: list[list[int]] | None = None
        self._gather_order = list(range(len(self.buckets)))[::-1]  # the layout is reversed: last bucket first
        self.probe = False  # device events around every gather wait (param_sync_exposed_ms)
        self._sync_ev: list[tuple] = []
        self._sync_steps = 0

    def enable_gather_overlap(self, stages: list[list[torch.Tensor]]) -> bool:
        """Let the next forward start while later buckets' parameters are still being all-gathered: the
        model calls ``wait_stage(i)`` before it reads stage i's parameters (``stages``: the trainable
        parameters grouped in forward order, as ``FlatAdamW.enable_overlap``), which waits only for the
        buckets that hold them.  The buckets are updated and gathered in the order of the stage that first
        needs them.  Returns False (nothing changed) when some bucket belongs to no stage."""
        where = {id(p): (o, _align(n)) for p, (o, n) in zip(self.params, self.offsets)}
        sb, order = [], []
        for group in stages:
            bs = sorted({b for o, n in (where[id(p)] for p in group if id(p) in where)
                         for b, (s, e) in enumerate(self.buckets) if o < e and o + n > s})
            sb.append(bs)
            order += [b for b in bs if b not in order]
        if sorted(order) != list(range(len(self.buckets))):
            return False
        self._stage_buckets, self._gather_order = sb, order
        return True

    def _wait(self, w):
        if self.probe and self.device.type == "cuda":
            e = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            e[0].record()
            w.wait()  # the current stream waits for the gather (device-side for RCCL)
            e[1].record()
            self._sync_ev.append(e)
        else:
            w.wait()

    def wait_stage(self, i: int):
        """The current stream waits for the parameter all-gathers of stage i's buckets."""
        if not self._pending or self._stage_buckets is None or i >= len(self._stage_buckets):
            return
        for b in self._stage_buckets[i]:
            w = self._pending.pop(b, None)
            if w is not None:
                self._wait(w)

    def join(self):
        """Every pending parameter all-gather is ordered before the current stream's next work (call before
        reading parameters outside the gated forward: checkpoints, exports, evaluation without gates)."""
        for b in list(self._pending):
            self._wait(self._pending.pop(b))

    def param_sync_exposed_ms(self, reset: bool = True) -> float | None:
        """Mean device time per optimizer step that streams spent waiting for the ZeRO-1 parameter
        all-gather (the part neither the rest of the update nor the next forward hid); None without
        probes.  Synchronises the device."""
        if not self.probe or not self._sync_steps:
            return None
        torch.cuda.synchronize(self.device)
        v = sum(a.elapsed_time(b) for a, b in self._sync_ev) / self._sync_steps
        if reset:
            self._sync_ev, self._sync_steps = [], 0
        return v

    def _launch_gather(self, b: int):
        import torch.distributed as dist

        s, e = self.buckets[b]
        lo, hi = self.shard_ranges[b]
        src = self.param_flat[lo:hi]
        # RCCL gathers in place (input == output + rank * count); gloo gets a private copy
        gloo = dist.get_backend(self.group) == "gloo"
        self._pending[b] = dist.all_gather_into_tensor(self.param_flat[s:e], src.clone() if gloo else src,
                                                       group=self.group, async_op=True)

    def _init_state(self):
        world, rank = self.world, self.rank
        self.shard_ranges: list[tuple[int, int]] = []  # owned [lo, hi) of param_flat per bucket
        self.shard_offsets: list[int] = []             # where each owned slice starts in the shard buffers
        n = 0
        for s, e in self.buckets:
            L = (e - s) // world
            self.shard_ranges.append((s + rank * L, s + (rank + 1) * L))
            self.shard_offsets.append(n)
            n += L
        self.shard_numel = n
        with torch.no_grad():
            self.master = torch.empty(n, dtype=torch.float32, device=self.device)
            for (lo, hi), o in zip(self.shard_ranges, self.shard_offsets):
                self.master[o:o + hi - lo].copy_(self.param_flat[lo:hi])
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=self.device)
        self.grad_shard = torch.zeros(n, dtype=self.grad_dtype, device=self.device)

    @torch.no_grad()
    def sync_master(self):
        self.join()
        for b, (lo, hi) in enumerate(self.shard_ranges):
            self.shard_view(b, self.master).copy_(self.param_flat[lo:hi])

    def shard_view(self, b: int, t: torch.Tensor) -> torch.Tensor:
        lo, hi = self.shard_ranges[b]
        o = self.shard_offsets[b]
        return t[o:o + hi - lo]

    @torch.no_grad()
    def step(self, lr: float | None = None):
        import torch.distributed as dist

        _linear.gradients_final()
        self.join()  # a bucket the last forward never gated on (the param_flat slices are rewritten below)
        lr = self.lr if lr is None else lr
        self.step_count += 1
        bump_param_generation()
        b1, b2 = self.betas
        g = self.grad_shard
        if use_hip(g) and self.dtype in (torch.bfloat16, torch.float32):
            stats = ext().grad_sumsq(g, 0.0, 1.0)  # local sum of squares of the owned slices
            dist.all_reduce(stats[0:1], group=self.group)
            norm = stats[0:1].sqrt() * self.grad_scale
            coef = torch.ones_like(norm)
            if self.max_grad_norm and self.max_grad_norm > 0:
                coef = torch.where(norm > self.max_grad_norm, self.max_grad_norm / (norm + 1e-6), coef)
            gscale = coef * self.grad_scale
            self.last_grad_norm = stats[0:1]
            for b in self._gather_order:  # each bucket's gather goes out right after its update
                lo, hi = self.shard_ranges[b]
                param = self.param_flat[lo:hi] if self.dtype == torch.bfloat16 else None
                ext().adamw_(param, self.shard_view(b, self.master), self.shard_view(b, self.exp_avg),
                             self.shard_view(b, self.exp_avg_sq), self.shard_view(b, g), lr, b1, b2, self.eps,
                             self.wd, self.step_count, gscale)
                if param is None:
                    self.param_flat[lo:hi].copy_(self.shard_view(b, self.master))
                self._launch_gather(b)
        else:
            gf = g.float() * self.grad_scale
            sq = (gf * gf).sum().reshape(1)
            dist.all_reduce(sq, group=self.group)
            self.last_grad_norm = sq / (self.grad_scale ** 2)
            norm = sq.sqrt()
            if self.max_grad_norm and self.max_grad_norm > 0:
                gf = gf * torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0)
            bc1, bc2 = 1 - b1 ** self.step_count, 1 - b2 ** self.step_count
            self.exp_avg.mul_(b1).add_(gf, alpha=1 - b1)
            self.exp_avg_sq.mul_(b2).addcmul_(gf, gf, value=1 - b2)
            self.master.mul_(1 - lr * self.wd)
            self.master.addcdiv_(self.exp_avg / bc1, (self.exp_avg_sq / bc2).sqrt_().add_(self.eps), value=-lr)
            for b in self._gather_order:
                lo, hi = self.shard_ranges[b]
                self.param_flat[lo:hi].copy_(self.shard_view(b, self.master))
                self._launch_gather(b)
        self._sync_steps += 1
        if self._stage_buckets is None:  # no gated forward follows: the update ends with the parameters
            self.join()

    def grad_norm(self) -> float:
        if self.last_grad_norm is None:
            return 0.0
        return float(self.last_grad_norm.float().sqrt().item()) * self.grad_scale

    def _gather_full(self, shard: torch.Tensor) -> torch.Tensor:
        """Full-layout fp32 copy (CPU) of a sharded state tensor; zeros in the padding."""
        import torch.distributed as dist

        out = torch.zeros(self.numel, dtype=torch.float32)
        for b, (s, e) in enumerate(self.buckets):
            full = torch.empty(e - s, dtype=torch.float32, device=self.device)
            dist.all_gather_into_tensor(full, self.shard_view(b, shard).contiguous(), group=self.group)
            out[s:e].copy_(full.cpu())
        return out

    def export_params(self) -> torch.Tensor:
        self.join()
        return super().export_params()

    @torch.no_grad()
    def import_params(self, compact: torch.Tensor):
        self.join()
        super().import_params(compact)

    def state_dict(self) -> dict:
        self.join()
        return {"format": "compact", "layout": self.layout(),
                **{k: self.compact(self._gather_full(getattr(self, k))) for k in ("master", "exp_avg", "exp_avg_sq")},
                "step": self.step_count, "lr": self.lr}

    @torch.no_grad()
    def load_state_dict(self, sd: dict):
        self.join()
        self._check_layout(sd)
        for name in ("master", "exp_avg", "exp_avg_sq"):
            full = self.expand_(sd[name], torch.zeros(self.numel, dtype=torch.float32))
            dst = getattr(self, name)
            for b in range(len(self.buckets)):
                lo, hi = self.shard_ranges[b]
                self.shard_view(b, dst).copy_(full[lo:hi])
        self.step_count = int(sd["step"])
        bump_param_generation()


def _fold_grad(p: torch.Tensor):
    """post-accumulate hook (fp32 grad buffer): main_grad += p.grad, then free p.grad.  Weights whose
    custom backward wrote main_grad itself return no gradient: the hook still fires, with p.grad None."""
    if p.grad is not None:
        p.main_grad.add_(p.grad)
        p.grad = None


def lr_at(step: int, base_lr: float, warmup: int, total: int, schedule: str = "cosine", min_ratio: float = 0.1) -> float:
    if warmup > 0 and step < warmup:
        return base_lr * (step + 1) / warmup
    if schedule == "constant" or total <= warmup:
        return base_lr
    t = min(1.0, (step - warmup) / max(1, total - warmup))
    if schedule == "linear":
        return base_lr * (1 - (1 - min_ratio) * t)
    return base_lr * (min_ratio + (1 - min_ratio) * 0.5 * (1 + math.cos(math.pi * t)))
