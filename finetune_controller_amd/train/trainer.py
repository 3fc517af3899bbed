"""The worker-side training loop: full fine-tune, LoRA and QLoRA for GPT-2 / Llama-3 / Mistral.

This is the piece the reference delegates to an opaque container image.  It
honours that image's contract with the controller:

* flags ``--dataset_path`` / ``--checkpoint_path`` (mounts ``/data/dataset`` and ``/data/artifacts``,
  ``/root/reference/app/models/examples/mnist.py:95-96``);
* ``metrics.csv`` appended every log interval (ingested by the monitor);
* log lines that contain ``Epoch`` (the UI log stream suppresses everything before the first one,
  ``/root/reference/app/utils/stream_logger.py:404-418``);
* flat, uniquely named artifacts matching the model's ``store_asset_patterns``;
* restart-safe: resumes from the newest ``checkpoint_step*.pt`` (backoffLimit restarts,
  ``/root/reference/app/jobs/kubeflow/PyTorchJobDeployer.py:183``) -- rank 0's choice, broadcast to
  ranks whose volume does not hold it (multi-node pods each have their own);
* failure detection: collective timeout, step watchdog, injectable faults (``utils.faults``).

Distributed: one process per GPU; gradients of the flat buffer are all-reduced in buckets
overlapped with backward (``parallel.ddp``); the optimizer averages via its device-side scale.
"""
from __future__ import annotations

import json
import logging
import os
import re
import time
from dataclasses import asdict, dataclass, field

import torch

from .. import ops
from ..models import LoRAConfig, build_model, get_config
from ..models import checkpoint as ckpt
from ..ops.linear import flush_fresh, join_wgrad_stream
from ..parallel import dist as pdist
from ..parallel.ddp import GradBucketer
from ..utils.faults import FaultInjector, StepWatchdog
from ..utils.metrics import MetricsCSV
from .data import EvalWindows, PackedTokenDataset, SyntheticTokens, Tokenizer
from .optim import FlatAdamW, ShardedFlatAdamW, lr_at

log = logging.getLogger("ftc.train")


@dataclass
class TrainConfig:
    model: str = "llama3-8b"
    method: str = "lora"  # lora | qlora | full
    lora_r: int = 16
    lora_alpha: float = 32.0
    lora_dropout: float = 0.0
    use_rslora: bool = False  # LoRA scale alpha / sqrt(r) instead of alpha / r
    lora_targets: list[str] = field(default_factory=lambda: ["q_proj", "k_proj", "v_proj", "o_proj", "gate_proj",
                                                              "up_proj", "down_proj"])
    batch_size: int = 4  # micro-batch per GPU (0: auto -- the HBM planner, utils/memplan.py)
    seq_len: int = 4096
    grad_accum: int = 1
    epochs: int = 1
    max_steps: int = 0  # 0 = epochs x steps_per_epoch (synthetic data: 100)
    lr: float = 2e-4
    warmup_steps: int = 10
    schedule: str = "cosine"
    weight_decay: float = 0.0
    max_grad_norm: float = 1.0
    seed: int = 1
    dataset_path: str = ""
    checkpoint_path: str = "./artifacts"
    log_interval: int = 10
    save_every: int = 0
    resume: bool = True
    synthetic: bool = False
    bucket_mb: float = 64.0
    comm_engine: str = "torch"  # torch | native
    # 1: ZeRO-1 (optimizer state sharded over data-parallel ranks, reduce-scatter grads + bf16 all-gather);
    # -1 (auto): ZeRO-1 for full fine-tuning on > 1 rank (exact fp32 reduction at 3/4 of an fp32
    # all-reduce's wire volume and 1/world of the AdamW state; docs/parallelism.md), else 0
    zero_stage: int = -1
    # Ulysses sequence parallelism: groups of `sp` consecutive ranks share the same sequences, each
    # holding 1/sp of every sequence's tokens (attention all-to-alls heads <-> tokens; parallel/sequence.py)
    sp: int = 1
    # gradient buffer / reduction dtype: fp32 | bf16 | auto (fp32 for full fine-tuning with gradient
    # accumulation or data parallelism -- summing 4+ bf16 micro-batch / rank gradients loses mantissa)
    grad_dtype: str = "auto"
    # the gradient reduction's dtype on the wire: "auto" = the gradient buffer's; "bf16" = an fp32 buffer
    # (exact local accumulation) reduced / reduce-scattered as bf16 (parallel.ddp: half the wire bytes)
    grad_wire: str = "auto"
    checkpoint_layers: bool | str = False  # "auto": only when the planned micro-batch needs it
    init_from: str = ""
    dtype: str = "auto"  # auto: bf16 on GPU, fp32 on CPU
    device: str = "auto"
    ce_chunk_rows: int = 4096
    save_model: bool = True
    timers: bool = False  # per-phase device timers (fwd/bwd/comm/optim) -> metrics.csv
    profile_steps: int = 0  # >0: torch.profiler chrome trace of that many steps -> trace_rank<r>.json
    graph: bool = False  # capture the whole training step in a hipGraph after 2 eager steps (1 GPU)
    eval_every: int = 0  # >0: held-out loss every that many optimizer steps (and after the last one)
    eval_batches: int = 4  # micro-batches per rank per evaluation
    eval_holdout: float = 0.01  # held-out share of the dataset's windows (>= 1: a window count)
    pack_documents: bool = False  # EOS-separated documents in a window attend only within themselves
    eos_id: int = -1  # -1: the dataset tokenizer's EOS (tokenizer.json, or the byte-level fallback's 2)
    completion_only: bool = False  # prompt/completion records: loss on the completion tokens only
    synthetic_doc_len: int = 0  # synthetic data: EOS every that many tokens (packed-document benchmarks)
    step_timeout_s: float = 0.0  # >0: exit 124 when no step / eval / save finishes for that long (FTC_STEP_TIMEOUT_S)
    # device events around the gradient-reduction wait of every step: the comm time backward did not
    # hide (``comm_exposed_ms``; bench.py turns it on for > 1 GPU)
    comm_probe: bool = False

    def lora_config(self) -> LoRAConfig | None:
        if self.method not in ("lora", "qlora"):
            return None
        return LoRAConfig(r=self.lora_r, alpha=self.lora_alpha, dropout=self.lora_dropout, use_rslora=self.use_rslora,
                          target_modules=list(self.lora_targets))


def resolve_zero_stage(zero_stage: int, method: str, world: int, sp: int = 1) -> int:
    """``zero_stage`` -1 (auto): ZeRO-1 for full fine-tuning with data parallelism.  Per rank per step
    it moves (n-1)/n (4 B + 2 B) per parameter -- an exact fp32 reduce-scatter plus a bf16 all-gather
    -- against 2 (n-1)/n 4 B for the fp32 all-reduce (42 vs 56 GB on 8 ranks for Llama-3-8B), and
    keeps 1/n of the 12 B/param AdamW state; adapters (MBs of gradients) keep the plain all-reduce."""
    if zero_stage >= 0:
        return zero_stage
    return 1 if (method == "full" and world > 1 and sp <= 1) else 0


class Trainer:
    def __init__(self, tc: TrainConfig):
        self.tc = tc
        self.info = pdist.init_distributed(tc.device)
        self.device = self.info.device
        torch.manual_seed(tc.seed)
        if tc.dtype == "auto":
            self.dtype = torch.bfloat16 if self.device.type == "cuda" else torch.float32
        else:
            self.dtype = {"bf16": torch.bfloat16, "fp32": torch.float32, "bfloat16": torch.bfloat16,
                          "float32": torch.float32}[tc.dtype]
        self.cfg = get_config(tc.model)
        if tc.seq_len > self.cfg.max_seq_len:
            self.cfg.max_seq_len = tc.seq_len
        self.lora = tc.lora_config()
        self.mem_plan = self._plan_memory()
        self.model = build_model(self.cfg, self.lora, device=self.device, dtype=self.dtype,
                                 checkpoint_layers=tc.checkpoint_layers)
        self.model.ce_chunk_rows = tc.ce_chunk_rows
        # sequence-parallel groups (collective: every rank creates every group); data-parallel index /
        # size = which sequences this rank's group trains on
        self.sp, self.dp_rank, self.dp_world = None, self.info.rank, self.info.world_size
        if tc.sp > 1:
            from ..parallel.sequence import make_seq_groups

            if not self.info.distributed:
                raise ValueError(f"sequence parallelism (sp={tc.sp}) needs WORLD_SIZE >= sp ranks")
            self.sp, self.dp_rank, self.dp_world = make_seq_groups(tc.sp, self.info.world_size, self.info.rank)
            if not hasattr(self.model, "set_sequence_parallel"):
                raise ValueError(f"model {tc.model} has no sequence-parallel attention")
            if tc.pack_documents:
                raise ValueError("packed documents are not supported with sequence parallelism")
            self.model.set_sequence_parallel(self.sp)
        self.model.init_weights(seed=tc.seed)
        if tc.init_from:
            n = ckpt.load_hf_checkpoint(self.model, tc.init_from)
            log.info("loaded %d tensors from %s", n, tc.init_from)
        if tc.method in ("lora", "qlora"):
            self.model.freeze_base()
        if tc.method == "qlora":
            from ..ops.nf4 import quantize_model_

            quantize_model_(self.model)
        self.model.train()
        self._memory_policy()
        # the loss is a per-micro-batch mean; summing grads over accum x world and scaling once
        # in the optimizer gives the global mean
        okw = dict(lr=tc.lr, weight_decay=tc.weight_decay, max_grad_norm=tc.max_grad_norm,
                   grad_scale=1.0 / (self.info.world_size * tc.grad_accum), grad_dtype=self._grad_dtype())
        trainable = [p for p in self.model.parameters() if p.requires_grad]
        self.zero_stage = resolve_zero_stage(tc.zero_stage, tc.method, self.info.world_size, tc.sp)
        if self.zero_stage >= 1 and self.info.distributed:
            esize = torch.finfo(self.dtype).bits // 8
            self.opt = ShardedFlatAdamW(trainable, self.info.world_size, self.info.rank,
                                        bucket_elems=max(1, int(tc.bucket_mb * 2 ** 20 / esize)), **okw)
        else:
            self.opt = FlatAdamW(trainable, **okw)
        if self.info.distributed:
            pdist.broadcast_params_([self.opt.param_flat], self.info)
            self.opt.sync_master()
            if tc.method == "full":
                pdist.broadcast_params_([p for p in self.model.parameters() if not p.requires_grad], self.info)
        self._overlap_update()
        tied = [self.model.lm_head] if self.cfg.tie_embeddings and tc.method == "full" else []
        if tc.grad_wire not in ("auto", "bf16", "bfloat16"):
            raise ValueError(f"grad_wire must be auto or bf16, not {tc.grad_wire!r}")
        wire = torch.bfloat16 if tc.grad_wire in ("bf16", "bfloat16") and self.opt.grad_flat.dtype == torch.float32 else None
        self.ddp = GradBucketer(self.opt, tc.bucket_mb, engine=tc.comm_engine, multi_use_params=tied, wire_dtype=wire)
        self._data = None
        self._eval_synth = None
        self.step = 0
        self.is_main = self.info.is_main
        self._timing: list[tuple] = []  # per-step (start, fwd, bwd, comm, optim) device events
        self._comm_ev: list[tuple] = []  # per-step (backward end, reduction complete) device events

    def _overlap_update(self):
        """Full fine-tuning: the AdamW update runs stage by stage on a side stream and the next forward
        waits per stage (``FlatAdamW.enable_overlap``), so the 8 B-parameter update (39 ms, HBM-bound)
        may share the chip with the first layers' GEMMs.  Off for
        adapters (a 0.3 ms update), ZeRO-1, hipGraph capture, per-phase timers and CPU runs.
        Opt-in (``FTC_OPT_OVERLAP=1``): measured neutral on Llama-3-8B (23,336 / 23,323 vs 23,332 /
        23,308 tok/s, profiles/r2/full_overlap/) -- the forward's GEMM and attention waves hold the
        register files of every CU, so the update's workgroups only run in the gaps between them."""
        import os

        tc = self.tc
        if isinstance(self.opt, ShardedFlatAdamW):
            # ZeRO-1: each bucket's parameter all-gather goes out right after its AdamW and the next
            # forward waits per layer for the buckets it reads (ShardedFlatAdamW.enable_gather_overlap);
            # FTC_ZERO_GATHER_OVERLAP=0 waits for every gather inside step()
            self.opt.probe = bool(tc.comm_probe and self.device.type == "cuda")
            if (os.environ.get("FTC_ZERO_GATHER_OVERLAP", "1") != "0" and not tc.graph
                    and hasattr(self.model, "param_stages") and self.opt.enable_gather_overlap(self.model.param_stages())):
                self.model.param_gate = self.opt.wait_stage
                log.info("ZeRO-1 parameter all-gather overlapped with the next forward (%d buckets)",
                         len(self.opt.buckets))
            return
        if (os.environ.get("FTC_OPT_OVERLAP", "0") != "1" or tc.method != "full" or type(self.opt) is not FlatAdamW
                or tc.graph or tc.timers or self.device.type != "cuda" or not hasattr(self.model, "param_stages")):
            return
        if self.opt.enable_overlap(self.model.param_stages()):
            opt = self.opt
            self.model.param_gate = opt.wait_stage
            log.info("optimizer update overlapped with the next forward (%d stages)", len(opt._stages))

    def _plan_memory(self):
        """``batch_size`` 0 / ``checkpoint_layers`` "auto": pick them from the model shape and this device's
        memory (utils.memplan; CPU runs plan against the host's free memory).  Fills in tc."""
        tc = self.tc
        if tc.batch_size > 0 and tc.checkpoint_layers != "auto":
            return None
        from ..utils import memplan

        if self.device.type == "cuda":
            dev_gb = torch.cuda.get_device_properties(self.device).total_memory / 1e9
        else:
            import psutil

            dev_gb = psutil.virtual_memory().available / 1e9
        p = memplan.plan(memplan.Dims.of(self.cfg), tc.method, tc.seq_len, dev_gb,
                         batch_size=tc.batch_size, checkpoint_layers=None if tc.checkpoint_layers == "auto"
                         else bool(tc.checkpoint_layers), world=self.info.world_size, zero_stage=tc.zero_stage,
                         grad_dtype=tc.grad_dtype, grad_accum=tc.grad_accum, lora_r=tc.lora_r, sp=tc.sp,
                         ce_chunk_rows=tc.ce_chunk_rows)
        tc.batch_size, tc.checkpoint_layers = p.batch_size, p.checkpoint_layers
        if self.info.is_main:
            log.info("memory plan: micro-batch %d x %d, checkpointing %s, %.1f of %.1f GB budget (%s)", p.batch_size,
                     tc.seq_len, "on" if p.checkpoint_layers else "off", p.peak_gb, p.budget_gb, p.parts_gb)
        return p

    def _grad_dtype(self) -> torch.dtype:
        tc = self.tc
        if tc.grad_dtype in ("fp32", "float32"):
            return torch.float32
        if tc.grad_dtype in ("bf16", "bfloat16") or self.dtype == torch.float32:
            return self.dtype
        if tc.grad_dtype != "auto":
            raise ValueError(f"grad_dtype must be auto, fp32 or bf16, not {tc.grad_dtype!r}")
        accumulating = tc.grad_accum > 1 or self.info.world_size > 1
        return torch.float32 if (tc.method == "full" and accumulating) else self.dtype

    def _memory_policy(self):
        """HBM budget decisions that depend on the model size: the TN backward GEMMs keep a transposed
        copy of every bf16 weight (+2 B/param); skip them when weights + copies would take more than
        45 % of the device (e.g. Llama-3-70B in bf16: 141 GB of weights on a 288 GB MI355X)."""
        if self.device.type != "cuda":
            return
        from ..ops.linear import set_tn_backward

        total = torch.cuda.get_device_properties(self.device).total_memory
        wbytes = sum(p.numel() * p.element_size() for p in self.model.parameters() if p.dim() == 2)
        on = 2 * wbytes <= 0.45 * total
        set_tn_backward(on)
        if not on and self.info.is_main:
            log.info("TN backward copies off: %.0f GB of 2-D weights on a %.0f GB device", wbytes / 1e9, total / 1e9)

    # ------------------------------------------------------------------ data
    def data(self):
        if self._data is None:
            tc = self.tc
            missing = not tc.dataset_path or not os.path.exists(tc.dataset_path) or not os.listdir(
                tc.dataset_path if os.path.isdir(tc.dataset_path) else os.path.dirname(tc.dataset_path))
            if missing and not tc.synthetic and os.environ.get("FTC_DATASET_EXPECTED") == "1":
                # the control plane attached a dataset to this job (k8s/manifest.py): an empty mount means the
                # download failed -- training on synthetic tokens would "complete" with a meaningless model
                raise FileNotFoundError(f"this job has a dataset but {tc.dataset_path!r} is missing or empty "
                                        "(did the dataset download fail?)")
            if tc.synthetic or missing:
                self._data = SyntheticTokens(self.cfg.vocab_size, tc.batch_size, tc.seq_len, self.device,
                                             seed=tc.seed + self.dp_rank, doc_len=tc.synthetic_doc_len,
                                             eos_id=self.eos_id() if tc.pack_documents else 2)
                self.steps_per_epoch = 100
            else:
                self._data = PackedTokenDataset(tc.dataset_path, self.cfg.vocab_size, tc.batch_size, tc.seq_len,
                                                self.device, self.dp_rank, self.dp_world, tc.seed,
                                                holdout=tc.eval_holdout if tc.eval_every > 0 else 0,
                                                eos_id=self.eos_id(), completion_only=tc.completion_only)
                self.steps_per_epoch = max(1, self._data.steps_per_epoch // tc.grad_accum)
            if self.sp is not None:  # this rank's contiguous 1/sp of every sequence of its group's batch
                from ..parallel.sequence import SeqShard

                self._data = SeqShard(self._data, self.sp)
        return self._data

    def eos_id(self) -> int | None:
        """The document separator when ``pack_documents`` is on."""
        tc = self.tc
        if not tc.pack_documents:
            return None
        if getattr(self, "_eos", None) is None:
            self._eos = tc.eos_id if tc.eos_id >= 0 else Tokenizer(
                tc.dataset_path if tc.dataset_path and os.path.exists(tc.dataset_path) else None,
                max(self.cfg.vocab_size, 259)).eos
        return self._eos

    def _batch(self, x, y, data):
        """(x, labels, segments, n_valid) of one micro-batch.  The data source masks the labels (packed
        documents: EOS inputs; completion-only: prompt tokens) and reports their count host-side
        (``last_n_valid``), so the loss normaliser needs no device sync; packed documents also get
        their segment bounds (attention stays inside a document, positions restart)."""
        eos = self.eos_id()
        seg = ops.segments_from_eos(x, eos) if eos is not None else None
        n_valid = getattr(data, "last_n_valid", None) if data is not None else None
        if n_valid is None and data is not None and eos is None and not self.tc.completion_only:
            n_valid = x.numel()  # nothing masked
        return x, y, seg, n_valid

    def total_steps(self) -> int:
        self.data()
        return self.tc.max_steps or self.tc.epochs * self.steps_per_epoch

    # ------------------------------------------------------------------ one step
    def graph_ok(self) -> bool:
        """Whole-step capture needs a step whose every launch argument is fixed: one rank (no
        collectives in the graph), the flat HIP AdamW (device-side schedule), a constant loss
        normaliser (no per-batch label masking) and no host-side timers."""
        tc = self.tc
        return (tc.graph and self.device.type == "cuda" and self.info.world_size == 1 and not tc.timers
                and type(self.opt) is FlatAdamW and ops.use_hip(self.opt.grad_flat) and not tc.pack_documents
                and not tc.completion_only)

    def train_step(self, lr: float) -> torch.Tensor:
        """fwd + bwd (+accum) + overlapped all-reduce + optimizer. Returns the loss (device tensor)."""
        if self.graph_ok():
            return self._graph_step(lr)
        return self._eager_step(lr)

    def _graph_step(self, lr: float) -> torch.Tensor:
        """Step through a captured hipGraph: launch-bound configurations (small models, short
        sequences) lose the host's per-kernel launch cost.  Two eager steps warm every cache (aug
        buffers, Wᵀ copies, hipBLASLt heuristics), the third is captured -- inputs copied into static
        buffers, lr / bias corrections read from the optimizer's device table -- and every step from
        then on is one graph launch.  Host-side bookkeeping the replay skips (optimizer step count,
        parameter generation for the eager caches) is advanced here."""
        from ..ops.linear import bump_param_generation

        tc = self.tc
        data = self.data()
        self._n_graph_calls = getattr(self, "_n_graph_calls", 0) + 1
        if self._n_graph_calls <= 2:
            return self._eager_step(lr)
        batches = [next(data) for _ in range(tc.grad_accum)]
        if getattr(self, "_graph", None) is None:
            self._gin = [(x.clone(), y.clone()) for x, y in batches]
            total = self.total_steps()
            lrs = [lr_at(s, tc.lr, tc.warmup_steps, total, tc.schedule) for s in range(self.step, max(total, self.step + 1))]
            self.opt.use_device_schedule(lrs + [lrs[-1]] * 1024)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._gout = self._eager_step(lr, inputs=self._gin)
            self._graph = g
            # the capture ran nothing: host state moved as if the step had run, the replay below runs it
            self.opt.step_count -= 1
        else:
            for (sx, sy), (x, y) in zip(self._gin, batches):
                sx.copy_(x, non_blocking=True)
                sy.copy_(y, non_blocking=True)
        self._graph.replay()
        self.opt.step_count += 1
        bump_param_generation()  # eager code after this step must re-read the updated adapters
        return self._gout.clone()

    def _eager_step(self, lr: float, inputs=None) -> torch.Tensor:
        tc = self.tc
        data = self.data()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)] if (tc.timers and self.device.type == "cuda") \
            else None
        if ev:
            ev[0].record()
        self.opt.zero_grad()
        total = None
        for micro in range(tc.grad_accum):
            x, y, seg, n_valid = self._batch(*(next(data) if inputs is None else inputs[micro]), data)
            self.ddp.armed = micro == tc.grad_accum - 1
            loss = self.model(x, y, n_valid=n_valid, segments=seg)
            if ev:
                ev[1].record()  # (last micro-batch's forward end)
            loss.backward()
            join_wgrad_stream()  # side-stream weight gradients (ops.linear, FTC_DW_STREAM) are complete
            total = loss.detach() if total is None else total + loss.detach()
        flush_fresh()  # skipped-zeroing weights this step never wrote (ops.linear first-write gradients)
        if ev:
            ev[2].record()
        probe = tc.comm_probe and self.device.type == "cuda" and self.ddp.enabled
        if probe:
            pe = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            pe[0].record()
        self.ddp.finish()  # device-side waits on the bucket all-reduces: the non-overlapped comm tail
        if probe:
            pe[1].record()
            self._comm_ev.append(pe)
        if ev:
            ev[3].record()
        self.opt.step(lr)
        if ev:
            ev[4].record()
            self._timing.append(tuple(ev))
        return total / tc.grad_accum

    # ------------------------------------------------------------------ evaluation
    def eval_batches(self):
        """Fixed held-out batches of this rank: the dataset's tail windows, or (synthetic data) a
        separate pool drawn from another seed."""
        data = self.data()
        if self.sp is not None:  # the group's ranks evaluate the same sequences, each its 1/P of them
            from ..parallel.sequence import shard_batch

            return (shard_batch(x, y, self.sp) for x, y in self._eval_full(data.inner))
        return self._eval_full(data)

    def _eval_full(self, data):
        if isinstance(data, PackedTokenDataset):
            return EvalWindows(data, self.tc.eval_batches).batches()
        if self._eval_synth is None:  # one pool per data-parallel replica (shared by an SP group)
            self._eval_synth = SyntheticTokens(self.cfg.vocab_size, self.tc.batch_size, self.tc.seq_len, self.device,
                                               seed=self.tc.seed + 7919 + self.dp_rank)
        self._eval_synth.i = 0  # the same batches every evaluation
        return (next(self._eval_synth) for _ in range(self.tc.eval_batches))

    def evaluate(self) -> float | None:
        """Mean next-token loss over the held-out batches of every rank (forward only, no gradients:
        the fused CE computes none under ``no_grad``).  None when there is nothing held out."""
        tc = self.tc
        was = self.model.training
        self.model.eval()
        # (sum of token losses, valid-token count) per rank, reduced over the world before dividing: the
        # token-weighted mean over every held-out token.  Sequence-parallel shards of one batch hold
        # unequal valid counts under label masking, so a mean of per-shard means would be biased.
        tot = torch.zeros(2, dtype=torch.float64, device=self.device)
        try:
            with torch.no_grad():
                for x, y in self.eval_batches():
                    x, y, seg, _ = self._batch(x, y, None)
                    lab = y.reshape(-1)
                    tot[0] += self.model(x, y, n_valid=1.0, segments=seg).double()  # normaliser 1: the sum
                    tot[1] += (lab != -100).sum().double()
        finally:
            self.model.train(was)
        pdist.all_reduce_mean_(tot, self.info)
        if float(tot[1]) == 0:
            return None
        return float(tot[0] / tot[1])

    def comm_exposed_ms(self, reset: bool = True) -> float | None:
        """Mean device time per step from the end of backward's last kernel to the completion of the
        gradient reduction (the part of the all-reduce / reduce-scatter backward did not hide), over
        the steps since the last reset; None without probes.  Synchronises the device."""
        if not self._comm_ev:
            return None
        torch.cuda.synchronize(self.device)
        v = sum(a.elapsed_time(b) for a, b in self._comm_ev) / len(self._comm_ev)
        if reset:
            self._comm_ev = []
        return v

    def param_sync_exposed_ms(self, reset: bool = True) -> float | None:
        """ZeRO-1: mean device time per step the streams waited for the parameter all-gather (None
        otherwise / without probes; ShardedFlatAdamW.param_sync_exposed_ms).  Synchronises the device."""
        f = getattr(self.opt, "param_sync_exposed_ms", None)
        return f(reset) if f is not None else None

    def _phase_ms(self) -> dict:
        """Mean fwd/bwd/comm/optim milliseconds of the steps since the last call (after a sync)."""
        if not self._timing:
            return {}
        acc = [0.0, 0.0, 0.0, 0.0]
        for ev in self._timing:
            for i in range(4):
                acc[i] += ev[i].elapsed_time(ev[i + 1])
        n = len(self._timing)
        self._timing = []
        return {k: round(v / n, 2) for k, v in zip(("fwd_ms", "bwd_ms", "comm_ms", "optim_ms"), acc)}

    # ------------------------------------------------------------------ loop
    def run(self) -> dict:
        tc = self.tc
        os.makedirs(tc.checkpoint_path, exist_ok=True)
        total = self.total_steps()
        start = 0
        st = self._resume_state() if tc.resume else None
        if st is not None:
            ckpt.apply_resume(st, self.opt)
            start = int(st["step"])
            self.data().load_state(st.get("data", {}))
            if self.is_main:
                log.info("resumed from checkpoint_step%d.pt", start)
        faults = FaultInjector.from_env(self.info.rank, tc.checkpoint_path)
        self.watchdog = watchdog = StepWatchdog.from_env(tc.step_timeout_s, self.info.rank)
        metrics = MetricsCSV(os.path.join(tc.checkpoint_path, "metrics.csv"), enabled=self.is_main,
                             resume=start > 0, resume_step=start if start > 0 else None)
        # tokens trained per optimizer step: every data-parallel replica's micro-batches (the ranks of a
        # sequence-parallel group share their sequences, so they count once)
        tok_per_step = tc.batch_size * tc.seq_len * tc.grad_accum * self.dp_world
        flops_tok = self.cfg.flops_per_token(tc.seq_len, lora=tc.method != "full")
        if self.is_main:
            n_train = self.opt.num_params()
            log.info("model=%s method=%s params=%.3fB trainable=%.2fM world=%d micro_batch=%d seq=%d accum=%d steps=%d",
                     self.cfg.name, tc.method, self.cfg.num_params() / 1e9, n_train / 1e6, self.info.world_size,
                     tc.batch_size, tc.seq_len, tc.grad_accum, total)
        last = {}
        sync = torch.cuda.synchronize if self.device.type == "cuda" else (lambda: None)
        sync()
        t0 = time.perf_counter()
        losses = []
        prof = None
        for step in range(start, total):
            faults.maybe_fire(step)
            lr = lr_at(step, tc.lr, tc.warmup_steps, total, tc.schedule)
            if tc.profile_steps and step == start + 2 and prof is None:
                from torch.profiler import ProfilerActivity, profile

                acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if self.device.type == "cuda" else [])
                prof = profile(activities=acts)
                prof.__enter__()
                prof_end = step + tc.profile_steps
            losses.append(self.train_step(lr))
            if prof is not None and step + 1 == prof_end:
                sync()
                prof.__exit__(None, None, None)
                prof.export_chrome_trace(os.path.join(tc.checkpoint_path, f"trace_rank{self.info.rank}.json"))
                prof = False
            self.step = step + 1
            watchdog.beat(f"step {self.step}")
            if self.step % tc.log_interval == 0 or self.step == total:
                sync()
                dt = time.perf_counter() - t0
                n = len(losses)
                # the global batch mean: each rank's loss is its micro-batches' mean (a sequence-parallel
                # rank's is its shard's sum over the batch's valid count / P), so the world mean is exact
                loss_t = pdist.all_reduce_mean_(torch.stack(losses).float().mean().reshape(1), self.info)
                loss_v = float(loss_t.item())
                step_ms = dt / n * 1000
                tps = tok_per_step * n / dt
                mem = torch.cuda.max_memory_allocated(self.device) / 1e9 if self.device.type == "cuda" else 0.0
                epoch = step // max(1, self.steps_per_epoch)
                last = {"epoch": epoch, "step": self.step, "loss": round(loss_v, 6), "lr": lr,
                        "tokens_per_sec": round(tps, 1), "step_time_ms": round(step_ms, 2),
                        "grad_norm": round(self.opt.grad_norm(), 6), "world_size": self.info.world_size,
                        "mem_gb": round(mem, 2),
                        "tflops_per_gpu": round(tps * flops_tok / self.info.world_size / 1e12, 1),
                        **self._phase_ms()}
                if self.is_main:
                    metrics.write(last)
                    # "Epoch" marks the start of the UI-visible log (LOG_STREAM_SEARCH_STRING)
                    print(f"Epoch {epoch} | step {self.step}/{total} | loss {loss_v:.4f} | lr {lr:.3e} | "
                          f"{tps:,.0f} tok/s | {step_ms:.1f} ms/step | grad_norm {last['grad_norm']:.4f} | "
                          f"mem {mem:.1f} GB", flush=True)
                losses = []
                t0 = time.perf_counter()
            if tc.eval_every and (self.step % tc.eval_every == 0 or self.step == total):
                ev_loss = self.evaluate()
                watchdog.beat(f"eval after step {self.step}")
                if ev_loss is not None:
                    last["eval_loss"] = round(ev_loss, 6)
                    if self.is_main:
                        metrics.write({"epoch": step // max(1, self.steps_per_epoch), "step": self.step,
                                       "eval_loss": last["eval_loss"], "world_size": self.info.world_size})
                        print(f"Epoch {step // max(1, self.steps_per_epoch)} | step {self.step}/{total} | "
                              f"eval_loss {ev_loss:.4f}", flush=True)
            if tc.save_every and self.step % tc.save_every == 0 and self.step < total:
                self.save_resume()
                watchdog.beat(f"checkpoint at step {self.step}")
        metrics.close()
        # training is over: the final save (a full-FT model or merged adapter can take minutes on rank 0)
        # and the barrier non-main ranks wait in get a phase limit of their own (FTC_SAVE_TIMEOUT_S,
        # default max(10 x the step limit, 1800 s)) -- long enough for the save, still an exit when a peer
        # hangs or dies there
        save_s = float(os.environ.get("FTC_SAVE_TIMEOUT_S", 0) or max(10 * watchdog.timeout_s, 1800.0))
        watchdog.phase("final save + barrier", save_s)
        if tc.save_model:
            self.save_artifacts()
        pdist.barrier(self.info)
        watchdog.close()
        return last

    def _resume_state(self) -> dict | None:
        """The resume state every rank starts from: rank 0's newest ``checkpoint_step*.pt`` (only rank
        0 writes them).  Ranks that see the same file read it; when any rank cannot (pod-local volumes
        of a multi-node job) rank 0 broadcasts the state instead."""
        rp = ckpt.latest_resume(self.tc.checkpoint_path)
        if not self.info.distributed:
            return ckpt.read_resume(rp) if rp else None
        import torch.distributed as dist

        dev = self.info.device if self.info.backend == "nccl" else torch.device("cpu")
        k = torch.tensor([ckpt.resume_step(rp) if rp else -1], dtype=torch.int64, device=dev)
        dist.broadcast(k, src=0)
        k = int(k.item())
        if k < 0:
            return None
        mine = os.path.join(self.tc.checkpoint_path, f"checkpoint_step{k}.pt")
        have = torch.tensor([int(os.path.exists(mine))], dtype=torch.int64, device=dev)
        dist.all_reduce(have, op=dist.ReduceOp.MIN)
        if int(have.item()):
            return ckpt.read_resume(mine)
        if self.is_main:
            log.info("checkpoint_step%d.pt is not on every rank's volume: broadcasting it", k)
        return pdist.broadcast_state(ckpt.read_resume(mine) if self.is_main else None, self.info)

    def _join_update(self):
        """An overlapped optimizer update (``_overlap_update``) is complete before host-side reads."""
        join = getattr(self.opt, "join", None)
        if join is not None:
            join()

    def save_resume(self):
        self._join_update()
        opt_state = self.opt.state_dict()  # collective under ZeRO-1 (gathers the sharded state)
        if not self.is_main:
            return
        p = os.path.join(self.tc.checkpoint_path, f"checkpoint_step{self.step}.pt")
        ckpt.save_resume(p, self.step, self.opt, self.data().state(), {"config": asdict(self.tc)},
                         opt_state=opt_state)
        # keep only the newest resume point (and no half-written .tmp left by a save a crash interrupted:
        # each is as large as a checkpoint)
        for old in os.listdir(self.tc.checkpoint_path):
            if re.fullmatch(r"checkpoint_step\d+\.pt(\.tmp)?", old) and old != os.path.basename(p):
                os.remove(os.path.join(self.tc.checkpoint_path, old))

    def save_artifacts(self) -> list[str]:
        self._join_update()
        if not self.is_main:
            return []
        out = self.tc.checkpoint_path
        if self.lora is not None:
            files = ckpt.save_adapter(self.model, out, self.cfg.name, self.lora)
        else:
            files = ckpt.save_full(self.model, out)
        runtime = {"kernels": ops.kernel_mode(), "device": str(self.device), "world_size": self.info.world_size,
                   "dist_backend": self.info.backend, "torch": torch.__version__,
                   "hip": getattr(torch.version, "hip", None),
                   "gpu": torch.cuda.get_device_name(self.device) if self.device.type == "cuda" else None}
        with open(os.path.join(out, "training_config.json"), "w") as f:
            json.dump({"train": asdict(self.tc), "model": self.cfg.to_dict(), "runtime": runtime}, f, indent=2,
                      default=str)
        return files

    def close(self):
        wd = getattr(self, "watchdog", None)
        if wd is not None:
            wd.close()
        if getattr(self, "opt", None) is not None:
            self._join_update()  # no collective may outlive the process group
        self.ddp.close()
        pdist.destroy(self.info)
