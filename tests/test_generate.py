"""KV-cache generation (models.generate): greedy decoding with the cache equals greedy decoding by
re-running the whole sequence, for several prompts of different lengths at once (sliding window
included); decode attention reference vs a direct softmax."""
import pytest
import torch

from finetune_controller_amd.models import LoRAConfig, build_model
from finetune_controller_amd.models.config import get_config
from finetune_controller_amd.models.generate import generate
from finetune_controller_amd.ops.decode import decode_attention_reference


def _naive_greedy(model, prompt, n):
    ids = list(prompt)
    out = []
    with torch.no_grad():
        for _ in range(n):
            logits = model(torch.tensor([ids]))
            t = int(logits[-1].argmax())
            out.append(t)
            ids.append(t)
    return out


@pytest.mark.parametrize("preset,lora", [("llama-tiny", False), ("mistral-tiny", False), ("llama-tiny", True)])
def test_kv_cache_greedy_matches_recompute(preset, lora):
    cfg = get_config(preset)
    torch.manual_seed(0)
    m = build_model(cfg, LoRAConfig(r=8, alpha=16) if lora else None, device="cpu", dtype=torch.float32)
    m.init_weights(seed=4)
    if lora:  # non-zero adapters so the LoRA path matters
        for layer in m.layers:
            for p in layer.lora.values():
                torch.nn.init.normal_(p.B, std=0.05)
    m.eval()
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(3, cfg.vocab_size, (n,), generator=g).tolist() for n in (5, 17, 60)]
    n_new = 12 if preset != "mistral-tiny" else 20  # mistral-tiny: window 64 < 60 + 20
    got = generate(m, prompts, max_new_tokens=n_new)
    for p, o in zip(prompts, got):
        assert o == _naive_greedy(m, p, n_new)


def test_generate_stops_at_eos_and_samples_reproducibly():
    cfg = get_config("llama-tiny")
    m = build_model(cfg, None, device="cpu", dtype=torch.float32)
    m.init_weights(seed=1)
    prompts = [[5, 6, 7], [9, 10]]
    greedy = generate(m, prompts, max_new_tokens=6)
    eos = greedy[0][2]
    cut = generate(m, prompts, max_new_tokens=6, eos_id=eos)
    assert cut[0] == greedy[0][:3]
    a = generate(m, prompts, max_new_tokens=6, temperature=0.8, top_p=0.9, seed=7)
    b = generate(m, prompts, max_new_tokens=6, temperature=0.8, top_p=0.9, seed=7)
    assert a == b and all(len(x) == 6 for x in a)


def test_decode_attention_reference():
    torch.manual_seed(0)
    B, L, H, KV, D = 3, 40, 4, 2, 16
    q = torch.randn(B, H * D)
    k, v = torch.randn(B, L, KV * D), torch.randn(B, L, KV * D)
    lens = torch.tensor([40, 7, 23], dtype=torch.int32)
    out = decode_attention_reference(q, k, v, lens, H, KV, D, 0.25, window=10)
    for b in range(B):
        n = int(lens[b])
        lo = max(0, n - 10)
        for h in range(H):
            kv = h // (H // KV)
            s = q[b, h * D:(h + 1) * D] @ k[b, lo:n, kv * D:(kv + 1) * D].T * 0.25
            o = s.softmax(-1) @ v[b, lo:n, kv * D:(kv + 1) * D]
            torch.testing.assert_close(out[b, h * D:(h + 1) * D], o, atol=1e-5, rtol=1e-5)


def test_generate_cli_loads_adapter(tmp_path, capsys):
    from finetune_controller_amd.models.generate import main
    from finetune_controller_amd.train.trainer import Trainer, TrainConfig

    tr = Trainer(TrainConfig(model="llama-tiny", method="lora", batch_size=1, seq_len=16, synthetic=True, max_steps=2,
                             checkpoint_path=str(tmp_path), resume=False, device="cpu", lr=1e-2, warmup_steps=0))
    tr.run()
    tr.close()
    capsys.readouterr()
    assert main(["--model", "llama-tiny", "--adapter", str(tmp_path), "--prompt", "hi", "--max-new-tokens", "4"]) == 0
    assert capsys.readouterr().out.startswith("hi")


def test_peft_target_forms_and_unknown_worker_targets():
    """Adapters from other tools name their targets as "all-linear", a list (possibly with modules this
    model has no LoRA slot for) or a regex; the trainer itself refuses a target it does not have."""
    import pytest

    from finetune_controller_amd.models.generate import peft_targets
    from finetune_controller_amd.models.lora import ALL_LINEAR, LoRAConfig

    assert peft_targets("all-linear") == ALL_LINEAR and peft_targets(None) == ALL_LINEAR
    assert peft_targets(["q_proj", "v_proj", "lm_head"]) == ["q_proj", "v_proj"]
    assert peft_targets(".*(q_proj|v_proj)$") == ["q_proj", "v_proj"]
    with pytest.raises(ValueError):
        peft_targets(["embed_tokens"])
    with pytest.raises(ValueError, match="unknown LoRA target"):
        LoRAConfig(target_modules=["q_proj", "qkv"])
