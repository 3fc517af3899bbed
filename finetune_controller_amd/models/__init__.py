"""Model families of the worker runtime: Llama-3 / Mistral trunk, GPT-2, LoRA / QLoRA adapters.

``config`` (presets and shapes) is plain Python; the torch modules load on first attribute access, so
the control plane (job specs, the HBM planner) can read model shapes without importing torch."""
from .config import PRESETS, ModelConfig, get_config  # noqa: F401

_LAZY = {"GPT2ForCausalLM": ".gpt2", "build_model": ".gpt2", "LlamaForCausalLM": ".llama", "ALL_LINEAR": ".lora",
         "LoRAConfig": ".lora", "LoRAPair": ".lora"}


def __getattr__(name):
    mod = _LAZY.get(name)
    if mod is None:
        raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
    import importlib

    return getattr(importlib.import_module(mod, __name__), name)
