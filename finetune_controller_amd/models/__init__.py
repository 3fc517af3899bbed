"""Model families of the worker runtime: Llama-3 / Mistral trunk, GPT-2, LoRA / QLoRA adapters."""
from .config import PRESETS, ModelConfig, get_config  # noqa: F401
from .gpt2 import GPT2ForCausalLM, build_model  # noqa: F401
from .llama import LlamaForCausalLM  # noqa: F401
from .lora import ALL_LINEAR, LoRAConfig, LoRAPair  # noqa: F401
