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

Layout: parameters are placed in REVERSE registration order (last layer first), i.e. in the order
backward produces their gradients, so the first DDP buckets become ready first.
"""
from __future__ import annotations

import math

import torch

from ..ops._backend import ext, use_hip
from ..ops.linear import bump_param_generation

ALIGN = 64  # elements: keeps every view 128-byte aligned for 16-byte vector access


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class FlatAdamW:
    def __init__(self, params, lr: float = 2e-4, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 max_grad_norm: float = 1.0, grad_scale: float = 1.0):
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
        self.params = list(reversed(plist))
        self.offsets: list[tuple[int, int]] = []
        off = 0
        for p in self.params:
            self.offsets.append((off, p.numel()))
            off += _align(p.numel())
        self.numel = off
        self.param_flat = torch.zeros(off, dtype=self.dtype, device=self.device)
        self.grad_flat = torch.zeros(off, dtype=self.dtype, device=self.device)
        with torch.no_grad():
            for p, (o, n) in zip(self.params, self.offsets):
                self.param_flat[o:o + n].copy_(p.detach().reshape(-1))
                p.data = self.param_flat[o:o + n].view_as(p)
                g = self.grad_flat[o:o + n].view_as(p)
                p.grad = g
                p.main_grad = g
        self.master = self.param_flat.float() if self.dtype != torch.float32 else self.param_flat
        self.exp_avg = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.exp_avg_sq = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.grad_scale = grad_scale  # e.g. 1/world_size when grads are summed by all-reduce
        self.step_count = 0
        self.last_grad_norm: torch.Tensor | None = None

    def num_params(self) -> int:
        return sum(n for _, n in self.offsets)

    def zero_grad(self):
        self.grad_flat.zero_()

    @torch.no_grad()
    def step(self, lr: float | None = None):
        lr = self.lr if lr is None else lr
        self.step_count += 1
        bump_param_generation()  # the update below rewrites param_flat in place
        b1, b2 = self.betas
        if use_hip(self.grad_flat) and self.dtype in (torch.bfloat16, torch.float32):
            stats = ext().grad_sumsq(self.grad_flat, self.max_grad_norm, self.grad_scale)
            self.last_grad_norm = stats[0:1]
            param = self.param_flat if self.dtype == torch.bfloat16 else None
            ext().adamw_(param, self.master, self.exp_avg, self.exp_avg_sq, self.grad_flat, lr, b1, b2, self.eps,
                         self.wd, self.step_count, stats[1:2])
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
        return {"master": self.master, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "step": self.step_count, "lr": self.lr, "numel": self.numel}

    @torch.no_grad()
    def load_state_dict(self, sd: dict):
        if int(sd["numel"]) != self.numel:
            raise ValueError("optimizer state does not match the parameter layout")
        self.master.copy_(sd["master"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.step_count = int(sd["step"])
        bump_param_generation()
        if self.master is not self.param_flat:
            self.param_flat.copy_(self.master)


def lr_at(step: int, base_lr: float, warmup: int, total: int, schedule: str = "cosine", min_ratio: float = 0.1) -> float:
    if warmup > 0 and step < warmup:
        return base_lr * (step + 1) / warmup
    if schedule == "constant" or total <= warmup:
        return base_lr
    t = min(1.0, (step - warmup) / max(1, total - warmup))
    if schedule == "linear":
        return base_lr * (1 - (1 - min_ratio) * t)
    return base_lr * (min_ratio + (1 - min_ratio) * 0.5 * (1 + math.cos(math.pi * t)))
