"""Parity with an independent implementation: Hugging Face ``transformers`` (importable here).

A tiny random model of each supported HF architecture is written with ``save_pretrained``
(safetensors), built in this framework from its ``config.json`` (``ModelConfig.from_hf_config``),
loaded through ``load_hf_checkpoint`` and compared on CPU in fp32: logits and the mean
next-token loss.  Covers Llama-3 (plain RoPE), Llama-3.1 ``rope_type: llama3`` frequency scaling,
Mistral sliding-window attention (sequence longer than the window) and GPT-2 (learned positions,
LayerNorm, GELU, tied head).  The loader must also refuse checkpoints with a missing or
mis-shaped tensor (models/checkpoint.py:load_hf_checkpoint).

Adapter-name parity with PEFT and NF4 layout parity with bitsandbytes stay *parity unpinned*:
neither library is importable in this image.
"""
import json
import os

import pytest
import torch

transformers = pytest.importorskip("transformers")

from finetune_controller_amd.models import build_model  # noqa: E402
from finetune_controller_amd.models.checkpoint import load_hf_checkpoint  # noqa: E402
from finetune_controller_amd.models.config import ModelConfig  # noqa: E402

_L31 = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
        "original_max_position_embeddings": 64}


def _hf_model(kind):
    torch.manual_seed(0)
    common = dict(vocab_size=211, hidden_size=64, intermediate_size=160, num_hidden_layers=2,
                  num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256,
                  rms_norm_eps=1e-5, tie_word_embeddings=False)
    if kind == "llama3":
        cfg = transformers.LlamaConfig(rope_theta=500000.0, **common)
        cls = transformers.LlamaForCausalLM
    elif kind == "llama3.1":
        cfg = transformers.LlamaConfig(rope_theta=500000.0, rope_scaling=dict(_L31), **common)
        cls = transformers.LlamaForCausalLM
    elif kind == "mistral":
        cfg = transformers.MistralConfig(rope_theta=10000.0, sliding_window=16, **common)
        cls = transformers.MistralForCausalLM
    else:
        cfg = transformers.GPT2Config(vocab_size=211, n_embd=64, n_layer=2, n_head=4, n_positions=128,
                                      n_inner=192, activation_function="gelu_new", resid_pdrop=0.0,
                                      embd_pdrop=0.0, attn_pdrop=0.0)
        cls = transformers.GPT2LMHeadModel
    cfg._attn_implementation = "eager"
    m = cls(cfg).float().eval()
    with torch.no_grad():  # non-trivial norms/biases so every parameter matters
        for name, p in m.named_parameters():
            if p.dim() == 1:
                p.add_(0.1 * torch.randn_like(p))
    return m


def _ours(path):
    with open(os.path.join(path, "config.json")) as f:
        cfg = ModelConfig.from_hf_config(json.load(f))
    m = build_model(cfg, None, device="cpu", dtype=torch.float32)
    n = load_hf_checkpoint(m, path)
    return m.eval(), n


@pytest.mark.parametrize("kind", ["llama3", "llama3.1", "mistral", "gpt2"])
def test_logits_and_loss_match_transformers(kind, tmp_path):
    hf = _hf_model(kind)
    hf.save_pretrained(tmp_path, safe_serialization=True)
    ours, n = _ours(str(tmp_path))
    assert n > 0
    B, S = 2, 40  # > the Mistral window (16): sliding-window masking is exercised
    ids = torch.randint(0, 211, (B, S), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        ref = hf(input_ids=ids).logits.float()
        got = ours(ids).reshape(B, S, -1).float()
        assert got.shape == ref.shape
        err = (got - ref).abs().max().item()
        assert err <= 2e-4 * max(1.0, ref.abs().max().item()), f"{kind}: max |dlogits| {err}"
        labels = ids.clone()
        ref_loss = torch.nn.functional.cross_entropy(ref[:, :-1].reshape(-1, ref.shape[-1]), labels[:, 1:].reshape(-1))
        shifted = torch.full_like(labels, -100)
        shifted[:, :-1] = labels[:, 1:]
        our_loss = ours(ids, shifted.reshape(-1))  # labels flattened like the [B*S, d] hidden rows
        our_loss = our_loss[0] if isinstance(our_loss, tuple) else our_loss
        assert abs(float(our_loss) - float(ref_loss)) < 1e-4, (kind, float(our_loss), float(ref_loss))


def test_loader_rejects_missing_and_misshaped_tensors(tmp_path):
    from safetensors.torch import load_file, save_file

    hf = _hf_model("llama3")
    hf.save_pretrained(tmp_path, safe_serialization=True)
    f = os.path.join(tmp_path, "model.safetensors")
    sd = load_file(f)
    # a partial checkpoint (one projection absent) must not silently train random weights
    part = {k: v for k, v in sd.items() if "layers.1.mlp.down_proj" not in k}
    save_file(part, f, metadata={"format": "pt"})
    with pytest.raises(ValueError, match="not found"):
        _ours(str(tmp_path))
    # a different architecture under the same names must be refused before any copy
    bad = dict(sd)
    bad["model.layers.0.self_attn.o_proj.weight"] = torch.zeros(64, 32)
    save_file(bad, f, metadata={"format": "pt"})
    with pytest.raises(ValueError, match="shape"):
        _ours(str(tmp_path))


@pytest.mark.parametrize("preset", ["llama-tiny", "mistral-tiny", "gpt2-tiny"])
def test_our_full_checkpoint_loads_in_transformers(preset, tmp_path):
    """The other direction: a full fine-tune export (save_full: safetensors + config.json) is a
    checkpoint ``transformers`` loads and runs to the same logits."""
    from finetune_controller_amd.models.checkpoint import save_full
    from finetune_controller_amd.models.config import get_config

    cfg = get_config(preset)
    m = build_model(cfg, None, device="cpu", dtype=torch.float32)
    m.init_weights(seed=3)
    m.eval()
    save_full(m, str(tmp_path))
    hf = transformers.AutoModelForCausalLM.from_pretrained(str(tmp_path), attn_implementation="eager", dtype=torch.float32).float().eval()
    ids = torch.randint(0, cfg.vocab_size, (2, 48), generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        ref = hf(input_ids=ids).logits.float()
        got = m(ids).reshape(2, 48, -1).float()
    err = (got - ref).abs().max().item()
    assert err <= 2e-4 * max(1.0, ref.abs().max().item()), f"{preset}: max |dlogits| {err}"
