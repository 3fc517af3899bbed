"""Walkthrough B (docs/models.md): a variant of a built-in LLM spec on the MI355X worker runtime.

Llama-3-8B LoRA with rank 64, 8k context and 2 GPUs per job.  Everything the built-in
``Llama3-8B-LoRA`` does -- the worker image, the ``train.cli`` command line, torchrun for more than
one GPU, ``amd.com/gpu`` requests -- is inherited; only defaults change.

Self-check::

    python docs/examples/custom_models/llama3_8b_lora_r64.py
"""
from typing import ClassVar

from pydantic import Field

from finetune_controller_amd.controlplane.spec.models.builtin import Llama3_8B_LoRA, LoRAArguments


class Llama3_8B_LoRA_R64(Llama3_8B_LoRA):
    name: str = "Llama3-8B-LoRA-r64-8k"
    description: str = "Llama-3-8B LoRA r=64, 8k tokens, 2 x MI355X data parallel"
    accelerator_count: int = Field(default=2, ge=1, description="MI355X GPUs per worker")
    promotion_path: str = Field(default="language/llama3-8b/lora-r64", description="s3 promotion prefix")
    training_arguments: LoRAArguments = LoRAArguments(lora_r=64, lora_alpha=128, seq_len=8192, batch_size=2)
    model_preset: ClassVar[str] = "llama3-8b"
    method: ClassVar[str] = "lora"


if __name__ == "__main__":
    m = Llama3_8B_LoRA_R64.model_validate(Llama3_8B_LoRA_R64())
    print(m.run_cmd())
