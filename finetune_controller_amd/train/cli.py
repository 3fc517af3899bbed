"""Worker entry point: ``python -m finetune_controller_amd.train.cli --model=llama3-8b --method=lora ...``.

This is the command the controller's PyTorchJob runs in container ``pytorch`` (see
``controlplane/spec/models/builtin.py``).  Flag names are the kebab-case forms of the spec's training
arguments plus the reference's mount contract ``--dataset_path`` / ``--checkpoint_path``
(``/root/reference/app/models/examples/mnist.py:94-96``).  Under ``torchrun`` one process per GPU
joins the RCCL process group from the injected ``RANK/WORLD_SIZE/MASTER_*`` variables.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

from .trainer import TrainConfig, Trainer


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="ftc-train", description="MI355X fine-tuning worker")
    ap.add_argument("--model", default="llama3-8b", help="preset name or HF config.json path")
    ap.add_argument("--method", default="lora", choices=["lora", "qlora", "full"])
    ap.add_argument("--lora-r", type=int, default=16)
    ap.add_argument("--lora-alpha", type=float, default=32.0)
    ap.add_argument("--lora-dropout", type=float, default=0.0)
    ap.add_argument("--use-rslora", action="store_true", help="LoRA scale alpha / sqrt(r)")
    ap.add_argument("--lora-targets", default="q_proj,k_proj,v_proj,o_proj,gate_proj,up_proj,down_proj")
    ap.add_argument("--batch-size", type=_int_or_auto, default=4,
                    help="micro-batch per GPU, or auto: the largest that fits 90 %% of the device (utils/memplan.py)")
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--grad-accum", type=int, default=1)
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--max-steps", type=int, default=0)
    ap.add_argument("--lr", type=float, default=2e-4)
    ap.add_argument("--warmup-steps", type=int, default=10)
    ap.add_argument("--schedule", default="cosine", choices=["cosine", "linear", "constant"])
    ap.add_argument("--weight-decay", type=float, default=0.0)
    ap.add_argument("--max-grad-norm", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--log-interval", type=int, default=10)
    ap.add_argument("--save-every", type=int, default=0)
    ap.add_argument("--checkpoint-layers", nargs="?", const="1", default="0", choices=["0", "1", "auto"],
                    help="activation checkpointing per decoder layer (auto: only when the micro-batch needs it)")
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--comm-engine", default="torch", choices=["torch", "native"])
    ap.add_argument("--sp", type=int, default=1,
                    help="Ulysses sequence parallelism degree: groups of SP ranks share each sequence")
    ap.add_argument("--zero-stage", type=int, default=-1, choices=[-1, 0, 1],
                    help="1: ZeRO-1 -- AdamW state sharded over the data-parallel ranks (reduce-scatter + all-gather); "
                         "-1 (auto): ZeRO-1 for full fine-tuning on > 1 GPU")
    ap.add_argument("--grad-dtype", default="auto", choices=["auto", "fp32", "bf16"],
                    help="gradient buffer / all-reduce dtype (auto: fp32 for full FT with accumulation or DP)")
    ap.add_argument("--grad-wire", default="auto", choices=["auto", "bf16"],
                    help="gradient reduction dtype on the wire (bf16: an fp32 gradient buffer reduced as bf16, "
                         "half the bytes; auto: the buffer's dtype)")
    ap.add_argument("--init-from", default="", help="HF safetensors checkpoint dir to fine-tune from")
    ap.add_argument("--synthetic", action="store_true", help="ignore the dataset; synthetic tokens")
    ap.add_argument("--no-resume", action="store_true")
    ap.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    ap.add_argument("--dtype", default="auto")
    ap.add_argument("--dataset_path", "--dataset-path", dest="dataset_path", default="/data/dataset")
    ap.add_argument("--checkpoint_path", "--checkpoint-path", dest="checkpoint_path", default="/data/artifacts")
    ap.add_argument("--timers", action="store_true", help="per-phase device timers (fwd/bwd/comm/optim) in metrics.csv")
    ap.add_argument("--profile-steps", type=int, default=0, help="torch.profiler chrome trace of N steps")
    ap.add_argument("--graph", action="store_true", help="capture the training step in a hipGraph (1 GPU)")
    ap.add_argument("--pack-documents", action="store_true",
                    help="EOS-separated documents in a window attend only within themselves (positions restart)")
    ap.add_argument("--completion-only", action="store_true",
                    help="prompt/completion records: no loss on prompt tokens")
    ap.add_argument("--eos-id", type=int, default=-1, help="document separator (-1: the dataset tokenizer's EOS)")
    ap.add_argument("--eval-every", type=int, default=0, help="held-out loss every N steps (0: off)")
    ap.add_argument("--eval-batches", type=int, default=4, help="micro-batches per rank per evaluation")
    ap.add_argument("--eval-holdout", type=float, default=0.01,
                    help="held-out share of the dataset windows (>= 1: a window count)")
    ap.add_argument("--step-timeout", type=float, default=0.0,
                    help="exit 124 when no step / eval / checkpoint finishes for this many seconds (0: off; "
                         "FTC_STEP_TIMEOUT_S overrides)")
    return ap


def _int_or_auto(v: str) -> int:
    """argparse type: a positive int, or "auto" -> 0 (the trainer plans it)."""
    if v == "auto":
        return 0
    n = int(v)
    if n < 1:
        raise argparse.ArgumentTypeError("batch size must be >= 1 or auto")
    return n


def config_from_args(a) -> TrainConfig:
    return TrainConfig(model=a.model, method=a.method, lora_r=a.lora_r, lora_alpha=a.lora_alpha,
                       lora_dropout=a.lora_dropout, use_rslora=a.use_rslora,
                       lora_targets=[t.strip() for t in a.lora_targets.split(",") if t.strip()],
                       batch_size=a.batch_size, seq_len=a.seq_len, grad_accum=a.grad_accum, epochs=a.epochs,
                       max_steps=a.max_steps, lr=a.lr, warmup_steps=a.warmup_steps, schedule=a.schedule,
                       weight_decay=a.weight_decay, max_grad_norm=a.max_grad_norm, seed=a.seed,
                       dataset_path=a.dataset_path, checkpoint_path=a.checkpoint_path, log_interval=a.log_interval,
                       save_every=a.save_every, resume=not a.no_resume, synthetic=a.synthetic, bucket_mb=a.bucket_mb,
                       comm_engine=a.comm_engine, zero_stage=a.zero_stage, grad_dtype=a.grad_dtype, grad_wire=a.grad_wire, sp=a.sp,
                       checkpoint_layers="auto" if a.checkpoint_layers == "auto" else a.checkpoint_layers == "1",
                       init_from=a.init_from,
                       dtype=a.dtype, device=a.device, timers=a.timers, profile_steps=a.profile_steps,
                       eval_every=a.eval_every, eval_batches=a.eval_batches, eval_holdout=a.eval_holdout,
                       pack_documents=a.pack_documents, eos_id=a.eos_id,
                       completion_only=a.completion_only, graph=a.graph,
                       step_timeout_s=a.step_timeout)


def main(argv=None) -> int:
    logging.basicConfig(level=os.environ.get("LOGLEVEL", "INFO").upper() if os.environ.get("LOGLEVEL") in
                        ("DEBUG", "INFO", "WARNING", "ERROR") else "INFO",
                        format="%(asctime)s %(name)s %(levelname)s %(message)s")
    a = build_parser().parse_args(argv)
    tr = Trainer(config_from_args(a))
    try:
        last = tr.run()
        if tr.is_main:
            print(f"Training complete: {last}", flush=True)
    finally:
        tr.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
