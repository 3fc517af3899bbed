"""Built-in fine-tune job specs.

* ``MNIST`` -- the reference's example (``/root/reference/app/models/examples/mnist.py:13-99``), kept so
  existing clients/frontends keep working; it still points at the external example image.
* MI355X specs for the BASELINE.json configs, all running this repository's worker runtime
  (``python -m finetune_controller_amd.train.cli``, see ``train/cli.py``) in the ROCm worker image:

  ==================  ===================================  =====================
  name                config                               resources
  ==================  ===================================  =====================
  GPT2-small-FT       GPT-2-small full fine-tune           1 CPU worker (plumbing)
  Llama3-8B-LoRA      Llama-3-8B LoRA bf16 (r16, all-lin)  amd.com/gpu x N
  Llama3-8B-Full      Llama-3-8B full FT, DDP over RCCL    amd.com/gpu x 8
  Mistral-7B-QLoRA    Mistral-7B QLoRA NF4                 amd.com/gpu x 1
  ==================  ===================================  =====================

Multi-GPU specs launch one process per GPU with torchrun inside the pod; with ``cluster_nodes > 1``
the Kubeflow operator's ``PET_*`` rendezvous variables are forwarded (one pod per node, one process
per GPU, RCCL over xGMI inside each node).
"""
from __future__ import annotations

from typing import Annotated, ClassVar, Literal

from pydantic import Field, field_validator

from ..finetuning import (BaseFineTuneModel, TrainingArguments, TrainingDataset, TrainingFramework,
                          TrainingResources, TrainingTask)

WORKER_IMAGE = "ghcr.io/finetune-controller-amd/worker-rocm:latest"


# ------------------------------------------------------------------ reference example (compat)
class MNISTConfig(TrainingArguments):
    """Model Params for MNIST Finetune Job"""

    batch_size: int = Field(default=64, description="Size of each batch during training")
    test_batch_size: int = Field(default=1000, description="Size of each batch during testing")
    epochs: int = Field(default=1, description="Number of epochs for training")
    lr: float = Field(default=1.0, description="Learning rate for the optimizer")
    gamma: float = Field(default=0.7, description="Learning rate step gamma for scheduler")
    no_cuda: bool = Field(default=False, description="Disable the GPU (use CPU instead)")
    seed: int = Field(default=1, description="Random seed for reproducibility")
    log_interval: int = Field(default=10, description="How many batches to wait before logging training status")
    save_model: bool = Field(default=False, description="Whether to save the trained model")


class MNIST(BaseFineTuneModel):
    """Finetune Job Spec for MNIST (external example image)"""

    name: str = "MNIST"
    inference_name: str | None = "MNIST"
    description: str = "Example MNIST model for fine-tuning"
    project_url: str = "https://github.com/acceleratedscience/model-foobar"
    image: str = "quay.io/brian_duenas/mnist:latest"
    command: list[str] = ["/bin/bash", "-c", "python mnist_training_script.py"]
    framework: TrainingFramework = TrainingFramework.PYTORCH
    task: TrainingTask = TrainingTask.CLASSIFICATION
    dataset_info: TrainingDataset = TrainingDataset(description="MNIST model does not expect a dataset",
                                                    dataset_required=False)
    resources: TrainingResources = TrainingResources(requests={"cpu": 4, "memory": "1Gi"},
                                                     limits={"cpu": 8, "memory": "2Gi"})
    # the reference's default of 0 (below ge=1, defaults are not validated) means "request no GPU"
    accelerator_count: int = Field(default=0, ge=1, description="Number of gpu devices to use for training per worker")
    promotion_path: str = Field(default="molecules/mnist/mnist_test", description="s3 promotion prefix")
    training_arguments: MNISTConfig = MNISTConfig()

    def run_cmd(self) -> list[str]:
        t = self.training_arguments
        args = []
        if t.no_cuda:
            args.append("--no-cuda")
        if t.save_model:
            args.append("--save-model")
        args += [f"--batch-size={t.batch_size}", f"--test-batch-size={t.test_batch_size}", f"--epochs={t.epochs}",
                 f"--lr={t.lr}", f"--seed={t.seed}", f"--log-interval={t.log_interval}", f"--gamma={t.gamma}"]
        return self.append_args(args)


class MNIST_MI355X(MNIST):
    """The reference's MNIST example on this repository's worker image: the same form and command line,
    run by ``finetune_controller_amd.train.mnist`` (one process per GPU under torchrun; CPU when
    ``accelerator_count`` is 0)."""

    name: str = "MNIST-MI355X"
    description: str = "Example MNIST classifier on the MI355X worker image"
    image: str = WORKER_IMAGE
    command: list[str] = ["/bin/bash", "-c", "python -m finetune_controller_amd.train.mnist"]
    store_asset_patterns: list[str] = Field(default=["*.json", "*.yaml", "*.csv", "*.pt", "*.ckpt"],
                                            description="Pattern match a list of files to store.")

    def run_cmd(self) -> list[str]:
        cmd = super().run_cmd()
        n = max(1, int(self.accelerator_count or 0))
        if n > 1:
            cmd[-1] = cmd[-1].replace("python -m", f"torchrun --standalone --nproc-per-node={n} -m", 1)
        return cmd


# ------------------------------------------------------------------ MI355X worker-runtime specs
class LMTrainingArguments(TrainingArguments):
    """Flags of ``finetune_controller_amd.train.cli`` exposed to the UI form."""

    # the int branch keeps its lower bound: 0 / negative values are rejected by the API, not by the
    # worker's argparse inside a restarting pod
    batch_size: Annotated[int, Field(ge=1)] | Literal["auto"] = Field(
        default=4, description="Micro-batch (sequences) per GPU, or auto: the largest that fits 90 % of the GPU's "
                               "HBM (utils/memplan.py), capped at 16k tokens")
    seq_len: int = Field(default=4096, ge=16, description="Tokens per sequence")
    grad_accum: int = Field(default=1, ge=1, description="Gradient accumulation steps")
    epochs: int = Field(default=1, ge=1, description="Passes over the dataset")
    max_steps: int = Field(default=0, ge=0, description="Stop after this many optimizer steps (0 = epochs)")
    lr: float = Field(default=2e-4, gt=0, description="Peak learning rate")
    warmup_steps: int = Field(default=10, ge=0, description="Linear warmup steps")
    schedule: Literal["cosine", "linear", "constant"] = Field(default="cosine", description="cosine | linear | constant")
    weight_decay: float = Field(default=0.0, ge=0, description="AdamW decoupled weight decay")
    max_grad_norm: float = Field(default=1.0, ge=0, description="Global grad-norm clip (0 = off)")
    seed: int = Field(default=1, description="Random seed")
    log_interval: int = Field(default=10, ge=1, description="Steps between metrics.csv rows / Epoch log lines")
    save_every: int = Field(default=0, ge=0, description="Resume checkpoint every N steps (0 = only at the end)")
    checkpoint_layers: bool | Literal["auto"] = Field(
        default=False, description="Activation checkpointing per decoder layer (auto: only when the micro-batch "
                                   "does not fit without it)")
    zero_stage: int = Field(default=-1, ge=-1, le=1,
                            description="1: ZeRO-1 -- AdamW state sharded over the data-parallel ranks; "
                                        "-1 (auto): ZeRO-1 for full fine-tuning on > 1 GPU")
    sp: int = Field(default=1, ge=1, le=64,
                    description="Ulysses sequence parallelism: groups of this many GPUs share each sequence "
                                "(long context; must divide the GPU count and the model's head counts)")
    grad_dtype: Literal["auto", "fp32", "bf16"] = Field(
        default="auto", description="Gradient buffer / all-reduce dtype (auto: fp32 for full FT with accumulation or DP)")
    grad_wire: Literal["auto", "bf16"] = Field(
        default="auto", description="Gradient reduction dtype on the wire (bf16: an fp32 buffer reduced as bf16, half "
                                    "the bytes on xGMI; auto: the buffer's dtype)")
    eval_every: int = Field(default=0, ge=0, description="Held-out loss every N steps (0 = off)")
    eval_batches: int = Field(default=4, ge=1, description="Micro-batches per GPU per evaluation")
    eval_holdout: float = Field(default=0.01, gt=0, description="Held-out share of the dataset (>= 1: windows)")
    pack_documents: bool = Field(default=False, description="Packed documents attend only within themselves")
    completion_only: bool = Field(default=False, description="prompt/completion data: loss on completions only")
    step_timeout: float = Field(default=0.0, ge=0,
                                description="Fail the worker (exit 124) when no step finishes for this many seconds "
                                            "(0 = off); the job then restarts from its last checkpoint")


_LORA_TARGETS = ("q_proj", "k_proj", "v_proj", "o_proj", "gate_proj", "up_proj", "down_proj")


class LoRAArguments(LMTrainingArguments):
    lora_r: int = Field(default=16, ge=1, le=256, description="LoRA rank")
    lora_alpha: float = Field(default=32.0, gt=0, description="LoRA alpha (scale = alpha / r)")
    lora_dropout: float = Field(default=0.0, ge=0.0, lt=1.0, description="Dropout on the adapter input")
    use_rslora: bool = Field(default=False, description="Rank-stabilised LoRA scale alpha / sqrt(r)")
    lora_targets: str = Field(default="q_proj,k_proj,v_proj,o_proj,gate_proj,up_proj,down_proj",
                              description="Comma-separated target modules")
    lr: float = Field(default=2e-4, gt=0, description="Peak learning rate")

    @field_validator("lora_targets")
    @classmethod
    def _known_targets(cls, v: str) -> str:
        # a typo would silently train fewer projections than asked (the worker has no such module)
        names = [t.strip() for t in v.split(",") if t.strip()]
        bad = [t for t in names if t not in _LORA_TARGETS]
        if not names or bad:
            raise ValueError(f"unknown LoRA target(s) {bad or v!r}; choose from {', '.join(_LORA_TARGETS)}")
        return ",".join(names)


class _WorkerSpec(BaseFineTuneModel):
    """Common run_cmd for specs that run this repository's trainer."""

    image: str = WORKER_IMAGE
    command: list[str] = ["/bin/bash", "-c", ""]
    framework: TrainingFramework = TrainingFramework.PYTORCH
    task: TrainingTask = TrainingTask.CAUSAL_LM
    store_asset_patterns: list[str] = Field(default=["*.json", "*.yaml", "*.csv", "*.pt", "*.ckpt", "*.safetensors"],
                                            description="Pattern match a list of files to store.")
    dataset_info: TrainingDataset = TrainingDataset(
        description="Optional: tokens (.bin uint16/uint32, .npy) or text (.jsonl with 'text', .txt, .csv). "
                    "Without a dataset the worker trains on synthetic tokens.", dataset_required=False)

    accelerator_memory_gb: float = Field(default=288.0, gt=0,
                                         description="HBM per GPU the auto batch planner sizes for (MI355X: 288 GB)")

    # subclass knobs (class-level, not form fields)
    model_preset: ClassVar[str] = "llama3-8b"
    method: ClassVar[str] = "lora"

    def memory_plan(self):
        """``utils.memplan.plan`` for this spec's model / method / world; None for a CPU job."""
        from finetune_controller_amd.models.config import get_config
        from finetune_controller_amd.utils import memplan

        t = self.training_arguments
        n = max(0, int(self.accelerator_count or 0)) * max(1, int(self.cluster_nodes or 1))
        if n == 0:
            return None
        ck = t.checkpoint_layers
        return memplan.plan(memplan.Dims.of(get_config(self.model_preset)), self.method, t.seq_len,
                            self.accelerator_memory_gb,
                            batch_size=0 if t.batch_size == "auto" else int(t.batch_size),
                            checkpoint_layers=None if ck == "auto" else bool(ck), world=n,
                            zero_stage=t.zero_stage, grad_dtype=t.grad_dtype, grad_accum=t.grad_accum,
                            lora_r=getattr(t, "lora_r", 16), sp=t.sp)

    def _launcher(self) -> str:
        n = max(1, int(self.accelerator_count))
        if n == 1 and self.cluster_nodes == 1:
            return "python -m finetune_controller_amd.train.cli"
        rdzv = ("--nnodes=${PET_NNODES:-1} --node-rank=${PET_NODE_RANK:-0} "
                "--master-addr=${PET_MASTER_ADDR:-127.0.0.1} --master-port=${PET_MASTER_PORT:-29500}"
                if self.cluster_nodes > 1 else "--standalone")
        return f"torchrun {rdzv} --nproc-per-node={n} -m finetune_controller_amd.train.cli"

    def run_cmd(self) -> list[str]:
        t = self.training_arguments
        vals = t.model_dump()
        if vals.get("batch_size") == "auto" or vals.get("checkpoint_layers") == "auto":
            # validated here against the spec's accelerator_memory_gb (memplan raises when nothing fits,
            # so an impossible job is refused at submission), but "auto" itself goes to the pod: the
            # worker re-plans against the real device's total_memory (Trainer._plan_memory), so a
            # spec that overstates the accelerator cannot render a micro-batch that OOMs
            self.memory_plan()
        args = [f"--model={self.model_preset}", f"--method={self.method}"]
        for k, v in vals.items():
            if isinstance(v, bool):
                if v:
                    args.append(f"--{k.replace('_', '-')}")
            elif k == "checkpoint_layers":  # "auto" (bool handled above)
                args.append("--checkpoint-layers=auto")
            else:
                args.append(f"--{k.replace('_', '-')}={v}")
        cmd = list(self.command)
        cmd[-1] = self._launcher()
        self_cmd = self.model_copy(update={"command": cmd})
        return BaseFineTuneModel.append_args(self_cmd, args)


class GPT2SmallFT(_WorkerSpec):
    """GPT-2-small full fine-tune on one CPU worker (BASELINE.json plumbing config)."""

    name: str = "GPT2-small-FT"
    inference_name: str | None = "GPT2-small"
    description: str = "GPT-2 small (124M) full fine-tune; CPU worker -- end-to-end plumbing of the controller"
    project_url: str = "https://huggingface.co/openai-community/gpt2"
    resources: TrainingResources = TrainingResources(requests={"cpu": 4, "memory": "8Gi"},
                                                     limits={"cpu": 8, "memory": "16Gi"})
    accelerator_count: int = Field(default=0, ge=1, description="CPU job: no GPU requested")
    promotion_path: str = Field(default="language/gpt2/finetune", description="s3 promotion prefix")
    model_preset: ClassVar[str] = "gpt2-small"
    method: ClassVar[str] = "full"
    training_arguments: LMTrainingArguments = LMTrainingArguments(batch_size=2, seq_len=256, lr=5e-5, max_steps=20)

    def run_cmd(self) -> list[str]:
        cmd = super().run_cmd()
        cmd[-1] += " --device=cpu"
        return cmd


class Llama3_8B_LoRA(_WorkerSpec):
    """Llama-3-8B LoRA (bf16) on MI355X -- the north-star config."""

    name: str = "Llama3-8B-LoRA"
    inference_name: str | None = "Llama3-8B"
    description: str = "Llama-3-8B LoRA fine-tune on AMD Instinct MI355X (HIP/CDNA4 kernels, RCCL data parallel)"
    project_url: str = "https://huggingface.co/meta-llama/Meta-Llama-3-8B"
    resources: TrainingResources = TrainingResources(requests={"cpu": 16, "memory": "128Gi"},
                                                     limits={"cpu": 32, "memory": "256Gi"})
    accelerator_count: int = Field(default=1, ge=1, description="MI355X GPUs per worker")
    promotion_path: str = Field(default="language/llama3-8b/lora", description="s3 promotion prefix")
    model_preset: ClassVar[str] = "llama3-8b"
    method: ClassVar[str] = "lora"
    training_arguments: LoRAArguments = LoRAArguments()


class Llama3_8B_LoRA_2GPU(Llama3_8B_LoRA):
    """Llama-3-8B LoRA data parallel over 2 x MI355X of one node (the Kueue multi-tenant config:
    four of these share an 8-GPU node; BASELINE.json configs[4])."""

    name: str = "Llama3-8B-LoRA-2GPU"
    description: str = "Llama-3-8B LoRA fine-tune, 2 x MI355X data parallel (RCCL all-reduce of the adapter grads)"
    accelerator_count: int = Field(default=2, ge=1, description="MI355X GPUs per worker")


class Llama3_8B_Full(_WorkerSpec):
    """Llama-3-8B full fine-tune, DDP over 8 x MI355X (RCCL all-reduce over xGMI)."""

    name: str = "Llama3-8B-Full"
    inference_name: str | None = "Llama3-8B"
    description: str = "Llama-3-8B full fine-tune, 8 x MI355X data parallel (bf16 weights, fp32 master/Adam)"
    project_url: str = "https://huggingface.co/meta-llama/Meta-Llama-3-8B"
    resources: TrainingResources = TrainingResources(requests={"cpu": 64, "memory": "512Gi"},
                                                     limits={"cpu": 128, "memory": "1024Gi"})
    accelerator_count: int = Field(default=8, ge=1, description="MI355X GPUs per worker")
    promotion_path: str = Field(default="language/llama3-8b/full", description="s3 promotion prefix")
    model_preset: ClassVar[str] = "llama3-8b"
    method: ClassVar[str] = "full"
    training_arguments: LMTrainingArguments = LMTrainingArguments(batch_size=2, lr=2e-5, checkpoint_layers=False)


class Mistral7B_QLoRA(_WorkerSpec):
    """Mistral-7B QLoRA (NF4 base, bf16 adapters) on one MI355X."""

    name: str = "Mistral-7B-QLoRA"
    inference_name: str | None = "Mistral-7B"
    description: str = "Mistral-7B QLoRA: NF4 base weights decoded on the fly for bf16 MFMA GEMMs"
    project_url: str = "https://huggingface.co/mistralai/Mistral-7B-v0.1"
    resources: TrainingResources = TrainingResources(requests={"cpu": 16, "memory": "64Gi"},
                                                     limits={"cpu": 32, "memory": "128Gi"})
    accelerator_count: int = Field(default=1, ge=1, description="MI355X GPUs per worker")
    promotion_path: str = Field(default="language/mistral-7b/qlora", description="s3 promotion prefix")
    model_preset: ClassVar[str] = "mistral-7b"
    method: ClassVar[str] = "qlora"
    training_arguments: LoRAArguments = LoRAArguments()


class Llama31_8B_LoRA(Llama3_8B_LoRA):
    """Llama-3.1-8B LoRA (Llama-3.1 RoPE frequency scaling; 128k positions)."""

    name: str = "Llama3.1-8B-LoRA"
    inference_name: str | None = "Llama3.1-8B"
    description: str = "Llama-3.1-8B LoRA fine-tune on one MI355X (long-context capable: 32k tokens without checkpointing)"
    project_url: str = "https://huggingface.co/meta-llama/Llama-3.1-8B"
    promotion_path: str = Field(default="language/llama3.1-8b/lora", description="s3 promotion prefix")
    model_preset: ClassVar[str] = "llama3.1-8b"


class Llama32_3B_LoRA(Llama3_8B_LoRA):
    """Llama-3.2-3B LoRA (tied embeddings, GQA 3:1)."""

    name: str = "Llama3.2-3B-LoRA"
    inference_name: str | None = "Llama3.2-3B"
    description: str = "Llama-3.2-3B LoRA fine-tune on one MI355X"
    project_url: str = "https://huggingface.co/meta-llama/Llama-3.2-3B"
    resources: TrainingResources = TrainingResources(requests={"cpu": 8, "memory": "64Gi"},
                                                     limits={"cpu": 16, "memory": "128Gi"})
    promotion_path: str = Field(default="language/llama3.2-3b/lora", description="s3 promotion prefix")
    model_preset: ClassVar[str] = "llama3.2-3b"


class Llama32_1B_LoRA(Llama32_3B_LoRA):
    """Llama-3.2-1B LoRA (tied embeddings, head_dim 64)."""

    name: str = "Llama3.2-1B-LoRA"
    inference_name: str | None = "Llama3.2-1B"
    description: str = "Llama-3.2-1B LoRA fine-tune on one MI355X"
    project_url: str = "https://huggingface.co/meta-llama/Llama-3.2-1B"
    promotion_path: str = Field(default="language/llama3.2-1b/lora", description="s3 promotion prefix")
    model_preset: ClassVar[str] = "llama3.2-1b"


class Llama3_70B_QLoRA(_WorkerSpec):
    """Llama-3-70B QLoRA on ONE MI355X (NF4 base in 288 GB of HBM)."""

    name: str = "Llama3-70B-QLoRA"
    inference_name: str | None = "Llama3-70B"
    description: str = "Llama-3-70B QLoRA on a single MI355X (NF4 base weights, bf16 adapters, ~4k tokens/s)"
    project_url: str = "https://huggingface.co/meta-llama/Meta-Llama-3-70B"
    resources: TrainingResources = TrainingResources(requests={"cpu": 16, "memory": "256Gi"},
                                                     limits={"cpu": 32, "memory": "512Gi"})
    accelerator_count: int = Field(default=1, ge=1, description="MI355X GPUs per worker")
    promotion_path: str = Field(default="language/llama3-70b/qlora", description="s3 promotion prefix")
    model_preset: ClassVar[str] = "llama3-70b"
    method: ClassVar[str] = "qlora"
    training_arguments: LoRAArguments = LoRAArguments(batch_size=2)


class Llama3_70B_LoRA(_WorkerSpec):
    """Llama-3-70B bf16 LoRA, data parallel over 8 x MI355X (all 141 GB of weights resident per GPU)."""

    name: str = "Llama3-70B-LoRA"
    inference_name: str | None = "Llama3-70B"
    description: str = "Llama-3-70B bf16 LoRA, 8 x MI355X data parallel (no weight sharding needed at 288 GB/GPU)"
    project_url: str = "https://huggingface.co/meta-llama/Meta-Llama-3-70B"
    resources: TrainingResources = TrainingResources(requests={"cpu": 64, "memory": "1024Gi"},
                                                     limits={"cpu": 128, "memory": "1536Gi"})
    accelerator_count: int = Field(default=8, ge=1, description="MI355X GPUs per worker")
    promotion_path: str = Field(default="language/llama3-70b/lora", description="s3 promotion prefix")
    model_preset: ClassVar[str] = "llama3-70b"
    method: ClassVar[str] = "lora"
    training_arguments: LoRAArguments = LoRAArguments(batch_size=1)


class Mistral7B_v03_LoRA(Llama3_8B_LoRA):
    """Mistral-7B-v0.3 LoRA (full attention, 32768 vocab)."""

    name: str = "Mistral-7B-v0.3-LoRA"
    inference_name: str | None = "Mistral-7B-v0.3"
    description: str = "Mistral-7B-v0.3 LoRA fine-tune on one MI355X"
    project_url: str = "https://huggingface.co/mistralai/Mistral-7B-v0.3"
    promotion_path: str = Field(default="language/mistral-7b-v0.3/lora", description="s3 promotion prefix")
    model_preset: ClassVar[str] = "mistral-7b-v0.3"


BUILTIN_MODELS = [MNIST, MNIST_MI355X, GPT2SmallFT, Llama3_8B_LoRA, Llama3_8B_LoRA_2GPU, Llama3_8B_Full, Mistral7B_QLoRA, Llama31_8B_LoRA,
                  Llama32_3B_LoRA, Llama32_1B_LoRA, Llama3_70B_QLoRA, Llama3_70B_LoRA, Mistral7B_v03_LoRA]
