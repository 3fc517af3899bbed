"""HBM planner: pick the micro-batch (and activation checkpointing) of a fine-tuning job from the
model shape and the device's memory -- ``batch_size: auto`` / ``checkpoint_layers: auto`` in the job
spec (``controlplane/spec/models/builtin.py``) and the worker CLI (``train/cli.py``).

The reference leaves batch sizing to the user's form (``/root/reference/app/models/base/finetuning.py:
28-34`` training arguments, ``:83-93`` resources / ``accelerator_count``); BASELINE.json's north star asks
for micro-batches sized for the 288 GB of HBM3E per MI355X.  Pure Python (no torch): the control plane
plans against the spec's ``accelerator_memory_gb`` to refuse a job that cannot fit, and passes ``auto``
on to the pod, where the worker plans against the real device's ``total_memory``.

Memory model (bytes), per GPU -- what the runtime of this repository allocates:

* frozen / trained weights: bf16 (2 B/param); QLoRA: NF4 trunk (0.5 B + a fp32 absmax per 64 =
  0.5625 B/param) with bf16 embeddings, norms and lm_head, plus the bf16 decode scratch of the largest
  projection (rows + transposed);
* transposed copies of the projection weights for the backward GEMMs (``ops.linear`` TN layout,
  +2 B/param) when the trainer's memory policy keeps them (2 x weights <= 45 % of the device);
* trainable state: bf16 params + grads (bf16, or fp32 under the ``grad_dtype`` auto policy: full FT
  with accumulation or data parallelism) + fp32 master + two fp32 AdamW moments; ZeRO-1 divides the
  master and moments by the data-parallel world;
* activations kept for backward, per token per layer: ``K_ACT x 2 B x (5 d + (H + 2 KV) hd + 3 F)`` --
  the residual stream and norm outputs, the qkv and attention outputs, gate / up and the SwiGLU
  product; with per-layer checkpointing only the layer inputs (h and the pending residual delta:
  ``4 d`` bytes per token per layer) plus ``K_CKPT`` layers' worth of recompute / backward transients;
* the chunked lm_head + cross-entropy (``ce_chunk_rows`` x vocab bf16) and a fixed allocator / library
  workspace slack.

Calibration (measured peaks on MI355X, ``torch.cuda.max_memory_allocated``; tests/test_memplan.py checks
every row within 10 %): Llama-3-8B LoRA 4 x 4096 107.7 GB, full FT 4 x 4096 218 GB, LoRA 1 x 32k 183 GB,
LoRA 1 x 64k with checkpointing 100 GB; Llama-3-70B LoRA bf16 1 x 4096 240 GB, QLoRA 2 x 4096 233 GB
(``BASELINE.md`` round-1 table, ``profiles/configs/``).
"""
from __future__ import annotations

from dataclasses import dataclass, field

GB = 1e9
K_ACT = 1.012         # fitted on Llama-3-8B LoRA 4 x 4096 (the implementation's extra tensors: LSE, LoRA tails)
K_CKPT = 3.4          # checkpointing: layers' worth of activations live at once (recompute + its backward)
SLACK_B = 2.0 * GB    # hipBLASLt workspace, RCCL buffers, allocator rounding
TN_POLICY_FRAC = 0.45  # trainer._memory_policy: TN copies only while 2 x weights <= 45 % of the device
MAX_FRAC = 0.9        # never plan past 90 % of the device
TARGET_TOKENS = 16384  # tokens per micro-batch at which the GEMMs and attention saturate 256 CUs (4 x 4096:
                       # 8 x 4096 measured no faster)


@dataclass
class Dims:
    """The shape facts the planner needs (``models.config.ModelConfig`` has them all)."""

    dim: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    ffn_dim: int
    vocab_size: int
    tie_embeddings: bool = False
    family: str = "llama"

    @classmethod
    def of(cls, cfg) -> "Dims":
        return cls(cfg.dim, cfg.n_layers, cfg.n_heads, cfg.n_kv_heads, cfg.ffn_dim, cfg.vocab_size,
                   bool(getattr(cfg, "tie_embeddings", False)), getattr(cfg, "family", "llama"))

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    def proj_params(self) -> int:
        """2-D projection weights of the trunk (the GEMM operands of every layer)."""
        d, hd, F = self.dim, self.head_dim, self.ffn_dim
        if self.family == "gpt2":
            return self.n_layers * (4 * d * d + 2 * F * d)
        return self.n_layers * ((self.n_heads + 2 * self.n_kv_heads) * hd * d + self.n_heads * hd * d + 3 * F * d)

    def embed_params(self) -> int:
        return self.vocab_size * self.dim * (1 if self.tie_embeddings else 2)

    def total_params(self) -> int:
        return self.proj_params() + self.embed_params() + (2 * self.n_layers + 1) * self.dim

    def act_elems_per_token_layer(self) -> int:
        d, hd, F = self.dim, self.head_dim, self.ffn_dim
        if self.family == "gpt2":
            return 5 * d + 3 * d + 2 * F
        return 5 * d + (self.n_heads + 2 * self.n_kv_heads) * hd + 3 * F

    def lora_params(self, r: int) -> int:
        """Adapters on all seven projections (q, k, v, o, gate, up, down)."""
        d, hd, F = self.dim, self.head_dim, self.ffn_dim
        q, kv = self.n_heads * hd, self.n_kv_heads * hd
        per = r * ((d + q) + 2 * (d + kv) + (q + d) + 2 * (d + F) + (F + d))
        return self.n_layers * per


@dataclass
class Plan:
    batch_size: int
    checkpoint_layers: bool
    peak_gb: float
    budget_gb: float
    tn_copies: bool
    parts_gb: dict = field(default_factory=dict)

    def as_args(self) -> dict:
        return {"batch_size": self.batch_size, "checkpoint_layers": self.checkpoint_layers}


def grad_bytes(method: str, grad_dtype: str, grad_accum: int, world: int) -> int:
    if grad_dtype in ("fp32", "float32"):
        return 4
    if grad_dtype in ("bf16", "bfloat16"):
        return 2
    return 4 if method == "full" and (grad_accum > 1 or world > 1) else 2


def estimate(dims: Dims, method: str, batch_size: int, seq_len: int, device_gb: float = 288.0, *,
             world: int = 1, zero_stage: int = -1, grad_dtype: str = "auto", grad_accum: int = 1, lora_r: int = 16,
             checkpoint_layers: bool = False, sp: int = 1, ce_chunk_rows: int = 4096) -> dict:
    """Peak bytes per GPU by component (floats, GB) for one configuration; ``total`` is their sum."""
    P, Pp = dims.total_params(), dims.proj_params()
    parts: dict[str, float] = {}
    if method == "qlora":
        parts["weights"] = Pp * 0.5625 + (P - Pp) * 2
        d, F = dims.dim, dims.ffn_dim
        parts["nf4_decode_scratch"] = 2 * 2 * 2 * F * d  # the largest projection (gate | up), rows + transposed
        tn = False
    else:
        parts["weights"] = 2.0 * P
        tn = 2 * (2.0 * Pp) <= TN_POLICY_FRAC * device_gb * GB
    if tn:
        parts["tn_copies"] = 2.0 * Pp
    zero = zero_stage if zero_stage >= 0 else (1 if method == "full" and world // max(1, sp) > 1 else 0)
    if method == "full":
        g = grad_bytes(method, grad_dtype, grad_accum, world)
        shard = max(1, world // max(1, sp)) if zero else 1
        parts["grads"] = g * P + (g * P / shard if zero else 0)
        parts["optimizer"] = 12.0 * P / shard  # fp32 master + exp_avg + exp_avg_sq
        # split-K fp32 partials of the down-projection dW (ops.linear.wgrad_mm, 2 token halves), one live
        # block per dW stream (main + side)
        parts["dw_split_scratch"] = 2 * (2 * 4.0 * dims.dim * dims.ffn_dim)
    else:
        A = dims.lora_params(lora_r)
        parts["adapters"] = 16.0 * A  # bf16 param + grad, fp32 master / m / v
    tokens = batch_size * seq_len / max(1, sp)
    per_tl = K_ACT * 2.0 * dims.act_elems_per_token_layer()
    if checkpoint_layers:
        parts["activations"] = tokens * dims.n_layers * 4.0 * dims.dim + K_CKPT * tokens * per_tl
    else:
        parts["activations"] = tokens * dims.n_layers * per_tl
    parts["lm_head_ce"] = 2.0 * min(ce_chunk_rows, tokens) * dims.vocab_size
    parts["slack"] = SLACK_B
    out = {k: v / GB for k, v in parts.items()}
    out["total"] = sum(parts.values()) / GB
    out["tn_copies_on"] = tn
    return out


def plan(dims: Dims, method: str, seq_len: int, device_gb: float = 288.0, *, batch_size: int = 0,
         checkpoint_layers: bool | None = None, target_tokens: int = TARGET_TOKENS, max_frac: float = MAX_FRAC,
         **kw) -> Plan:
    """The largest micro-batch (at most ``target_tokens`` tokens, at least one sequence) that fits
    ``max_frac`` of the device, without activation checkpointing when it fits, else with it.
    ``batch_size`` > 0 / ``checkpoint_layers`` not None pin that choice.  Raises ValueError when not even
    one sequence fits (more GPUs with sequence parallelism, or a shorter ``seq_len``)."""
    budget = max_frac * device_gb
    sp = max(1, int(kw.get("sp", 1)))
    cap = max(1, target_tokens // max(1, seq_len // sp)) if batch_size <= 0 else batch_size
    modes = [checkpoint_layers] if checkpoint_layers is not None else [False, True]
    for ck in modes:
        sizes = [batch_size] if batch_size > 0 else list(range(cap, 0, -1))
        for b in sizes:
            e = estimate(dims, method, b, seq_len, device_gb, checkpoint_layers=ck, **kw)
            if e["total"] <= budget:
                parts = {k: round(v, 2) for k, v in e.items() if k not in ("total", "tn_copies_on")}
                return Plan(b, ck, round(e["total"], 1), round(budget, 1), bool(e["tn_copies_on"]), parts)
    e = estimate(dims, method, max(1, batch_size), seq_len, device_gb, checkpoint_layers=modes[-1], **kw)
    raise ValueError(f"{method} at seq_len {seq_len}: {e['total']:.0f} GB per GPU even at micro-batch "
                     f"{max(1, batch_size)}{' with checkpointing' if modes[-1] else ''} > {budget:.0f} GB "
                     f"({max_frac:.0%} of {device_gb:.0f} GB): use sequence parallelism (sp) or a shorter seq_len")
