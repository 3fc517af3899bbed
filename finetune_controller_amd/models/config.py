"""Model architecture presets for the worker runtime.

The reference ships only an opaque MNIST image (``/root/reference/app/models/examples/mnist.py:48-53``);
the fine-tune targets named by BASELINE.json are built here from their public configs
(SURVEY.md §2.3 "[external]" shapes):

* ``llama3-8b``  -- d 4096, 32 layers, 32 q heads / 8 kv heads x 128, FFN 14336, vocab 128256, RoPE 5e5
* ``mistral-7b`` -- same trunk, vocab 32000, RoPE 1e4, sliding window 4096 (v0.1)
* ``gpt2-small`` -- d 768, 12 layers, 12 heads x 64, FFN 3072, vocab 50257, LayerNorm + GELU, learned positions

plus Llama-3.1 / 3.2 / 70B and Mistral v0.3 members of the same trunk, and ``*-tiny`` variants of
each family used by CPU tests and the FakeCluster e2e job.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field


@dataclass
class ModelConfig:
    family: str  # "llama" (llama/mistral trunk) or "gpt2"
    vocab_size: int
    dim: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    ffn_dim: int
    max_seq_len: int = 8192
    rope_theta: float = 10000.0
    rope_scaling: dict | None = None
    norm_eps: float = 1e-5
    sliding_window: int = 0  # 0 = full causal
    tie_embeddings: bool = False
    name: str = ""
    extra: dict = field(default_factory=dict)

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    def num_params(self) -> int:
        d, D, F = self.dim, self.head_dim, self.ffn_dim
        if self.family == "gpt2":
            per = 4 * d + (3 * d * d + 3 * d) + (d * d + d) + (F * d + F) + (d * F + d)
            emb = self.vocab_size * d + self.max_seq_len * d
            return emb + self.n_layers * per + 2 * d
        qkv = (self.n_heads + 2 * self.n_kv_heads) * D * d
        per = 2 * d + qkv + self.n_heads * D * d + 3 * F * d
        emb = self.vocab_size * d * (1 if self.tie_embeddings else 2)
        return emb + self.n_layers * per + d

    def flops_per_token(self, seq_len: int, lora: bool) -> float:
        """Model FLOPs per trained token (matmuls + attention), fwd+bwd.

        Frozen-base LoRA skips the weight-gradient GEMMs of the base (2 instead of 3 passes).
        """
        d, D, F = self.dim, self.head_dim, self.ffn_dim
        if self.family == "gpt2":
            mm = self.n_layers * (3 * d * d + d * d + 2 * F * d) + self.vocab_size * d
        else:
            mm = self.n_layers * ((self.n_heads + 2 * self.n_kv_heads) * D * d + self.n_heads * D * d + 3 * F * d)
            mm += self.vocab_size * d
        attn = self.n_layers * 2 * self.n_heads * D * seq_len  # causal: half of 4*S*H*D
        passes = 2.0 if lora else 3.0
        return 2.0 * mm * passes + attn * (1.0 + 2.5)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    def to_hf_config(self) -> dict:
        """config.json in the Hugging Face layout (written next to full-FT checkpoints)."""
        if self.family == "gpt2":
            return {"architectures": ["GPT2LMHeadModel"], "model_type": "gpt2", "vocab_size": self.vocab_size,
                    "n_embd": self.dim, "n_layer": self.n_layers, "n_head": self.n_heads,
                    "n_positions": self.max_seq_len, "n_inner": self.ffn_dim, "layer_norm_epsilon": self.norm_eps,
                    "tie_word_embeddings": True}
        mt = "mistral" if self.sliding_window else "llama"
        cfg = {"architectures": ["MistralForCausalLM" if mt == "mistral" else "LlamaForCausalLM"], "model_type": mt,
               "vocab_size": self.vocab_size, "hidden_size": self.dim, "num_hidden_layers": self.n_layers,
               "num_attention_heads": self.n_heads, "num_key_value_heads": self.n_kv_heads,
               "intermediate_size": self.ffn_dim, "max_position_embeddings": self.max_seq_len,
               "rope_theta": self.rope_theta, "rms_norm_eps": self.norm_eps, "hidden_act": "silu",
               "tie_word_embeddings": self.tie_embeddings, "torch_dtype": "bfloat16"}
        if self.sliding_window:
            cfg["sliding_window"] = self.sliding_window
        if self.rope_scaling:
            cfg["rope_scaling"] = self.rope_scaling
        # transformers >= 5 reads RoPE only from "rope_parameters" (the top-level keys above serve 4.x)
        cfg["rope_parameters"] = {"rope_type": "default", **(self.rope_scaling or {}), "rope_theta": self.rope_theta}
        return cfg

    @classmethod
    def from_hf_config(cls, cfg: dict, name: str = "") -> "ModelConfig":
        mt = cfg.get("model_type", "llama")
        if mt == "gpt2":
            d = cfg["n_embd"]
            return cls("gpt2", cfg["vocab_size"], d, cfg["n_layer"], cfg["n_head"], cfg["n_head"],
                       cfg.get("n_inner") or 4 * d, cfg.get("n_positions", 1024), norm_eps=cfg.get("layer_norm_epsilon", 1e-5),
                       tie_embeddings=True, name=name or "gpt2")
        # transformers >= 5 writes RoPE settings as one "rope_parameters" dict (theta + scaling);
        # older configs carry top-level "rope_theta" / "rope_scaling"
        rp = dict(cfg.get("rope_parameters") or {})
        theta = float(rp.pop("rope_theta", cfg.get("rope_theta", 10000.0)))
        scaling = cfg.get("rope_scaling")
        if scaling is None and rp.get("rope_type", "default") != "default":
            scaling = rp
        if scaling and scaling.get("rope_type", scaling.get("type", "default")) == "default":
            scaling = None
        hd = cfg.get("head_dim")
        if hd and hd * cfg["num_attention_heads"] != cfg["hidden_size"]:
            raise ValueError(f"head_dim {hd} x {cfg['num_attention_heads']} heads != hidden_size {cfg['hidden_size']}: "
                             "decoupled head_dim is not supported")
        return cls("llama", cfg["vocab_size"], cfg["hidden_size"], cfg["num_hidden_layers"], cfg["num_attention_heads"],
                   cfg.get("num_key_value_heads", cfg["num_attention_heads"]), cfg["intermediate_size"],
                   cfg.get("max_position_embeddings", 8192), theta, scaling,
                   cfg.get("rms_norm_eps", 1e-5), cfg.get("sliding_window") or 0,
                   cfg.get("tie_word_embeddings", False), name=name or mt)


_L31 = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
        "original_max_position_embeddings": 8192}

PRESETS: dict[str, ModelConfig] = {
    "llama3-8b": ModelConfig("llama", 128256, 4096, 32, 32, 8, 14336, 8192, 500000.0, name="llama3-8b"),
    "mistral-7b": ModelConfig("llama", 32000, 4096, 32, 32, 8, 14336, 32768, 10000.0, sliding_window=4096,
                              name="mistral-7b"),
    "gpt2-small": ModelConfig("gpt2", 50257, 768, 12, 12, 12, 3072, 1024, tie_embeddings=True, name="gpt2-small"),
    # further members of the Llama trunk (public configs): Llama-3.1 frequency scaling, Llama-3.2's tied
    # embeddings and head_dim 64 (1B) / 24-head GQA 3:1 (3B), the 80-layer 70B (QLoRA fits one
    # 288 GB MI355X), Mistral v0.3 (full attention, 32768 vocab)
    "llama3.1-8b": ModelConfig("llama", 128256, 4096, 32, 32, 8, 14336, 131072, 500000.0, name="llama3.1-8b",
                               rope_scaling=_L31),
    "llama3.2-1b": ModelConfig("llama", 128256, 2048, 16, 32, 8, 8192, 131072, 500000.0, tie_embeddings=True,
                               name="llama3.2-1b", rope_scaling={**_L31, "factor": 32.0}),
    "llama3.2-3b": ModelConfig("llama", 128256, 3072, 28, 24, 8, 8192, 131072, 500000.0, tie_embeddings=True,
                               name="llama3.2-3b", rope_scaling={**_L31, "factor": 32.0}),
    "llama3-70b": ModelConfig("llama", 128256, 8192, 80, 64, 8, 28672, 8192, 500000.0, name="llama3-70b"),
    "mistral-7b-v0.3": ModelConfig("llama", 32768, 4096, 32, 32, 8, 14336, 32768, 1000000.0, name="mistral-7b-v0.3"),
    # test-sized members of each family (same code paths, seconds on CPU)
    "llama-tiny": ModelConfig("llama", 512, 128, 2, 4, 2, 256, 512, 500000.0, name="llama-tiny"),
    "mistral-tiny": ModelConfig("llama", 384, 128, 2, 4, 2, 256, 512, 10000.0, sliding_window=64, name="mistral-tiny"),
    "gpt2-tiny": ModelConfig("gpt2", 515, 128, 2, 4, 4, 512, 256, tie_embeddings=True, name="gpt2-tiny"),
    # Llama-3 attention geometry (head_dim 128, GQA 2:1) at toy width: exercises every HIP kernel in smoke()
    "llama-smoke": ModelConfig("llama", 1024, 512, 2, 4, 2, 1024, 1024, 500000.0, name="llama-smoke"),
    # a 1-layer member of the exact Llama-3-8B width, for kernel/GEMM-shape smoke tests on the GPU
    "llama3-8b-1l": ModelConfig("llama", 128256, 4096, 1, 32, 8, 14336, 8192, 500000.0, name="llama3-8b-1l"),
}


def get_config(name_or_path: str) -> ModelConfig:
    if name_or_path in PRESETS:
        return dataclasses.replace(PRESETS[name_or_path])
    with open(name_or_path) as f:
        return ModelConfig.from_hf_config(json.load(f))
