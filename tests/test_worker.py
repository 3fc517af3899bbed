"""Worker runtime on CPU: op semantics (torch path = the numerics oracle of the HIP kernels), LoRA /
QLoRA layers, checkpoint formats (PEFT adapter, HF shards), resume, data formats, and data-parallel
gradient equivalence over gloo with 2 processes."""
import json
import math
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from finetune_controller_amd import ops
from finetune_controller_amd.models import LoRAConfig, build_model, get_config
from finetune_controller_amd.models import checkpoint as ckpt
from finetune_controller_amd.models.lora import merge_pair_into
from finetune_controller_amd.ops import nf4
from finetune_controller_amd.train.data import EvalWindows, PackedTokenDataset, load_token_array, load_tokens_and_mask
from finetune_controller_amd.utils.metrics import read_metrics_csv
from finetune_controller_amd.train.optim import FlatAdamW, lr_at
from finetune_controller_amd.train.trainer import TrainConfig, Trainer


def test_lora_linear_grads_match_autograd():
    torch.manual_seed(0)
    x = torch.randn(6, 16, requires_grad=True)
    W = torch.randn(12, 16)
    A = torch.randn(4, 16, requires_grad=True)
    B = torch.randn(12, 4, requires_grad=True)
    blocks = [(0, 8, 0, 2), (8, 12, 2, 4)]
    mask = torch.zeros(12, 4)
    for r0, r1, c0, c1 in blocks:
        mask[r0:r1, c0:c1] = 1
    Bm = (B * mask).detach().requires_grad_(True)
    y = ops.lora_linear(x, W, A, Bm, 0.5, blocks=blocks)
    x2, A2, B2 = x.detach().clone().requires_grad_(True), A.detach().clone().requires_grad_(True), \
        Bm.detach().clone().requires_grad_(True)
    ref = x2 @ W.t() + 0.5 * (x2 @ A2.t()) @ (B2 * mask).t()
    torch.testing.assert_close(y, ref)
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g)
    torch.testing.assert_close(x.grad, x2.grad)
    torch.testing.assert_close(A.grad, A2.grad)
    torch.testing.assert_close(Bm.grad, B2.grad)
    assert (Bm.grad * (1 - mask)).abs().max() == 0  # off-diagonal blocks stay structural zeros


class _PadIdentity(torch.autograd.Function):
    """Hands ``x`` on as a column view of a row-padded buffer and the gradient likewise (what the
    RMSNorm / SwiGLU / flash producers do on the GPU)."""

    @staticmethod
    def forward(ctx, x, pad):
        ctx.pad = pad
        buf = torch.full((x.shape[0], x.shape[1] + pad), float("nan"))
        buf[:, :x.shape[1]] = x
        return buf[:, :x.shape[1]]

    @staticmethod
    def backward(ctx, g):
        return g, None


class _PadGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, pad):
        ctx.pad = pad
        return y.clone()

    @staticmethod
    def backward(ctx, g):
        buf = torch.full((g.shape[0], g.shape[1] + ctx.pad), float("nan"))
        buf[:, :g.shape[1]] = g
        return buf[:, :g.shape[1]], None


def test_augmented_lora_gemms_match_two_gemm_path():
    """ops.linear augmented path: y = [x | xA^T][W | sB]^T and dx = [dy | dyB][W ; sA] computed in
    the producers' spare columns (NaN-filled here, so any read of an unwritten column fails)."""
    from finetune_controller_amd.ops.linear import AugWeight

    torch.manual_seed(0)
    T, K, N, R = 10, 16, 24, 8
    aw = AugWeight(N, K, R, dtype=torch.float32)
    aw.W.copy_(torch.randn(N, K))
    W = torch.nn.Parameter(aw.W, requires_grad=False)
    assert aw.owns(W)
    A = torch.randn(R, K, requires_grad=True)
    B = torch.randn(N, R, requires_grad=True)
    x = torch.randn(T, K, requires_grad=True)
    y = _PadGrad.apply(ops.lora_linear(_PadIdentity.apply(x, aw.Rp), W, A, B, 0.5, aug=aw), aw.Rp)
    x2, A2, B2 = (t.detach().clone().requires_grad_(True) for t in (x, A, B))
    ref = x2 @ W.detach().clone().t() + 0.5 * (x2 @ A2.t()) @ B2.t()
    torch.testing.assert_close(y, ref)
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g)
    for a_, b_ in ((x.grad, x2.grad), (A.grad, A2.grad), (B.grad, B2.grad)):
        assert torch.isfinite(a_).all()
        torch.testing.assert_close(a_, b_)


@pytest.mark.parametrize("packed", [False, True])
def test_augmented_lora_direct_main_grad_and_refresh_across_steps(packed):
    """A/B homed in FlatAdamW's flat buffers: their grads are accumulated in place (beta=1 GEMMs, grad
    -ready hook fired, nothing returned to autograd), and the augmented operands are re-copied once
    per optimizer step -- the second forward must see the updated A/B."""
    from finetune_controller_amd.ops import linear as lin

    torch.manual_seed(0)
    T, K, N, R = 10, 16, 24, 8
    blocks = [(0, 16, 0, 4), (16, 24, 4, 8)] if packed else None  # packed projection: block-diagonal B
    aw = lin.AugWeight(N, K, R, dtype=torch.float32)
    aw.W.copy_(torch.randn(N, K))
    W = torch.nn.Parameter(aw.W, requires_grad=False)
    A = torch.nn.Parameter(torch.randn(R, K))
    B = torch.nn.Parameter(torch.randn(N, R))
    if packed:
        with torch.no_grad():
            mask = torch.zeros(N, R)
            for r0, r1, c0, c1 in blocks:
                mask[r0:r1, c0:c1] = 1
            B.mul_(mask)
    opt = FlatAdamW([A, B], lr=1e-1, max_grad_norm=0.0)
    ready = []
    lin.set_grad_ready_hook(ready.append)
    try:
        for step in range(2):
            x = torch.randn(T, K, requires_grad=True)
            y = _PadGrad.apply(ops.lora_linear(_PadIdentity.apply(x, aw.Rp), W, A, B, 0.5, blocks=blocks, aug=aw),
                               aw.Rp)
            x2, A2, B2 = (t.detach().clone().requires_grad_(True) for t in (x, A, B))
            ref = x2 @ W.detach().clone().t() + 0.5 * (x2 @ A2.t()) @ (B2 * mask if packed else B2).t()
            torch.testing.assert_close(y, ref)
            g = torch.randn_like(y)
            opt.zero_grad()
            ready.clear()
            y.backward(g)
            ref.backward(g)
            assert {id(p) for p in ready} == {id(A), id(B)}
            torch.testing.assert_close(x.grad, x2.grad)
            torch.testing.assert_close(A.main_grad, A2.grad)
            torch.testing.assert_close(B.main_grad, B2.grad)
            if packed:
                assert (B.main_grad * (1 - mask)).abs().max() == 0 and (B.detach() * (1 - mask)).abs().max() == 0
            opt.step()
    finally:
        lin.set_grad_ready_hook(None)


def test_fused_ce_matches_reference():
    torch.manual_seed(0)
    h = torch.randn(37, 16, requires_grad=True)
    W = torch.randn(50, 16, requires_grad=True)
    lab = torch.randint(0, 50, (37,))
    lab[5] = -100
    loss = ops.fused_linear_cross_entropy(h, W, lab, chunk_rows=8)
    h2, W2 = h.detach().clone().requires_grad_(True), W.detach().clone().requires_grad_(True)
    ref = ops.cross_entropy_reference(h2, W2, lab)
    torch.testing.assert_close(loss, ref, atol=1e-5, rtol=1e-5)
    (loss * 2).backward()
    (ref * 2).backward()
    torch.testing.assert_close(h.grad, h2.grad, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(W.grad, W2.grad, atol=1e-5, rtol=1e-4)


def test_rope_and_attention_reference_paths():
    torch.manual_seed(0)
    B, S, H, KV, D = 2, 16, 4, 2, 16
    qkv = torch.randn(B * S, (H + 2 * KV) * D)
    tab = ops.RotaryTable(D, 64, 10000.0)
    rot = ops.apply_rope_packed(qkv, tab, H, KV, D, S)
    # rotation preserves per-pair norms; v untouched
    n0 = qkv[:, :(H + KV) * D].view(B * S, H + KV, 2, D // 2).pow(2).sum(2)
    n1 = rot[:, :(H + KV) * D].view(B * S, H + KV, 2, D // 2).pow(2).sum(2)
    torch.testing.assert_close(n0, n1, atol=1e-4, rtol=1e-4)
    assert torch.equal(rot[:, (H + KV) * D:], qkv[:, (H + KV) * D:])
    out = ops.attention_packed(qkv, B, S, H, KV, D, True, 0)
    ref = ops.attention_reference(qkv, B, S, H, KV, D, True, 0)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-4)
    outw = ops.attention_packed(qkv, B, S, H, KV, D, True, 4)
    refw = ops.attention_reference(qkv, B, S, H, KV, D, True, 4)
    torch.testing.assert_close(outw, refw, atol=1e-5, rtol=1e-4)


def test_llama_lora_starts_as_identity_and_merges():
    cfg = get_config("llama-tiny")
    torch.manual_seed(0)
    base = build_model(cfg, None, dtype=torch.float32)
    base.init_weights(seed=3)
    lora = build_model(cfg, LoRAConfig(r=4, alpha=8), dtype=torch.float32)
    lora.load_state_dict({k: v for k, v in base.state_dict().items()}, strict=False)
    x = torch.randint(0, cfg.vocab_size, (2, 32))
    with torch.no_grad():
        torch.testing.assert_close(lora(x), base(x))  # B = 0
        for layer in lora.layers:
            for p in layer.lora.values():
                for _, _, B_s in p.segment_tensors():  # diagonal blocks only (off-blocks are structural 0)
                    B_s.normal_(0, 0.1)
        y_lora = lora(x)
        for layer in lora.layers:
            for name, p in layer.lora.items():
                merge_pair_into(layer.base_weight(name).data, p, +1.0)
                p.B.zero_()
        torch.testing.assert_close(lora(x), y_lora, atol=1e-4, rtol=1e-4)


def test_adapter_export_peft_names_and_roundtrip(tmp_path):
    cfg = get_config("llama-tiny")
    lc = LoRAConfig(r=4, alpha=8, target_modules=["q_proj", "v_proj", "down_proj"])
    m = build_model(cfg, lc, dtype=torch.float32)
    m.init_weights()
    for layer in m.layers:
        for p in layer.lora.values():
            for _, _, B_s in p.segment_tensors():
                B_s.data.normal_()
    files = ckpt.save_adapter(m, str(tmp_path), "llama-tiny", lc)
    assert {os.path.basename(f) for f in files} == {"adapter_model.safetensors", "adapter_model.pt", "adapter_config.json"}
    assert not [f for f in os.listdir(tmp_path) if f.endswith(".tmp")]  # written as .tmp, renamed into place
    sd = ckpt.adapter_state_dict(m)
    k = "base_model.model.model.layers.0.self_attn.q_proj.lora_A.weight"
    assert k in sd and sd[k].shape == (4, cfg.dim)
    assert sd["base_model.model.model.layers.1.mlp.down_proj.lora_B.weight"].shape == (cfg.dim, 4)
    assert not any("k_proj" in key for key in sd)
    conf = json.load(open(tmp_path / "adapter_config.json"))
    assert conf["peft_type"] == "LORA" and conf["r"] == 4 and conf["lora_alpha"] == 8
    m2 = build_model(cfg, lc, dtype=torch.float32)
    n = ckpt.load_adapter(m2, str(tmp_path))
    assert n == 2 * 3
    # an adapter that does not fit the model is refused, not loaded in part
    m3 = build_model(cfg, LoRAConfig(r=4, alpha=8, target_modules=["q_proj", "v_proj"]), dtype=torch.float32)
    with pytest.raises(ValueError, match="down_proj.lora_A.weight has no LoRA slot"):
        ckpt.load_adapter(m3, str(tmp_path))
    m4 = build_model(cfg, LoRAConfig(r=4, alpha=8, target_modules=["q_proj", "v_proj", "down_proj", "o_proj"]),
                     dtype=torch.float32)
    for layer in m4.layers:  # stale values in the slot the adapter does not train
        layer.lora["o_proj"].B.data.fill_(1.0) if "o_proj" in layer.lora else None
    assert ckpt.load_adapter(m4, str(tmp_path)) == 2 * 3  # a model with MORE slots: the extra one is zeroed
    assert all(float(layer.lora[n].B.abs().sum()) == 0 for layer in m4.layers for n in layer.lora
               if "o_proj" in layer.lora[n].names)
    # a truncated file (layer 1 lost its q_proj pair while keeping v / down) is refused
    trunc = {k: v for k, v in sd.items() if "layers.1.self_attn.q_proj" not in k}
    with pytest.raises(ValueError, match="LoRA segments missing"):
        ckpt.load_adapter(m2, ckpt.save_file(trunc, str(tmp_path / "t.safetensors")) or str(tmp_path / "t.safetensors"))
    # a partial-layer PEFT adapter (layers_to_transform = [0]) loads; layer 1 contributes nothing
    only0 = {k: v for k, v in sd.items() if ".layers.0." in k}
    os.makedirs(tmp_path / "l0")
    ckpt.save_file(only0, str(tmp_path / "l0" / "adapter_model.safetensors"))
    json.dump({**conf, "layers_to_transform": [0]}, open(tmp_path / "l0" / "adapter_config.json", "w"))
    m5 = build_model(cfg, lc, dtype=torch.float32)
    for layer in m5.layers:
        for p in layer.lora.values():
            for _, _, B_s in p.segment_tensors():
                B_s.data.fill_(1.0)
    assert ckpt.load_adapter(m5, str(tmp_path / "l0")) == 3
    assert all(float(B_s.abs().sum()) == 0 for p in m5.layers[1].lora.values() for _, _, B_s in p.segment_tensors())
    assert all(float(B_s.abs().sum()) > 0 for p in m5.layers[0].lora.values() for _, _, B_s in p.segment_tensors())
    with pytest.raises(ValueError, match="LoRA segments missing"):  # it claims layer 1 but does not carry it
        ckpt.load_adapter(m5, str(tmp_path / "l0"), layers_to_transform=[0, 1])
    part = {k: v for k, v in sd.items() if "layers.1.mlp.down_proj.lora_B" not in k}
    with pytest.raises(ValueError, match="no down_proj.lora_B partner"):
        ckpt.load_adapter(m2, ckpt.save_file(part, str(tmp_path / "p.safetensors")) or str(tmp_path / "p.safetensors"))
    for a, b in zip(m.layers, m2.layers):
        for name in a.lora:
            torch.testing.assert_close(a.lora[name].B.to(torch.bfloat16).float(), b.lora[name].B)


def test_full_checkpoint_hf_roundtrip(tmp_path):
    for preset in ("llama-tiny", "gpt2-tiny"):
        cfg = get_config(preset)
        m = build_model(cfg, None, dtype=torch.float32)
        m.init_weights(seed=1)
        files = ckpt.save_full(m, str(tmp_path / preset))
        idx = json.load(open(tmp_path / preset / "model.safetensors.index.json"))
        if preset == "llama-tiny":
            assert "model.layers.0.self_attn.k_proj.weight" in idx["weight_map"]
        else:
            assert "transformer.h.0.attn.c_attn.weight" in idx["weight_map"]
        m2 = build_model(cfg, None, dtype=torch.float32)
        n = ckpt.load_hf_checkpoint(m2, str(tmp_path / preset))
        assert n == len(idx["weight_map"])
        x = torch.randint(0, cfg.vocab_size, (1, 16))
        with torch.no_grad():
            torch.testing.assert_close(m(x), m2(x))
        assert any(f.endswith("config.json") for f in files)


def test_nf4_cpu_quantization():
    torch.manual_seed(0)
    w = torch.randn(64, 128) * 0.05
    q = nf4.NF4Weight.quantize(w)
    assert q.packed.numel() == w.numel() // 2 and q.absmax_q.dtype == torch.uint8
    deq = q.dequantize(torch.float32)
    rel = (deq - w).abs().max() / w.abs().max()
    assert rel < 0.2
    # codebook round-trip of exact code points is lossless up to the double-quantised absmax
    assert nf4.NF4_CODE.shape == (16,) and nf4.NF4_CODE[7] == 0.0


def test_qlora_model_trains_on_cpu(tmp_path):
    tc = TrainConfig(model="llama-tiny", method="qlora", batch_size=2, seq_len=32, synthetic=True, max_steps=3,
                     log_interval=1, checkpoint_path=str(tmp_path), resume=False, lr=1e-2, warmup_steps=0,
                     device="cpu", dtype="fp32")
    tr = Trainer(tc)
    assert tr.model.layers[0].qweights and tr.model.layers[0].wqkv.numel() == 0
    last = tr.run()
    tr.close()
    assert last["step"] == 3 and math.isfinite(last["loss"])


def test_flat_adamw_matches_torch():
    torch.manual_seed(0)
    p1 = torch.nn.Parameter(torch.randn(10, 3))
    p2 = torch.nn.Parameter(torch.randn(7))
    q1, q2 = torch.nn.Parameter(p1.detach().clone()), torch.nn.Parameter(p2.detach().clone())
    opt = FlatAdamW([p1, p2], lr=1e-2, weight_decay=0.1, max_grad_norm=0.0)
    ref = torch.optim.AdamW([q1, q2], lr=1e-2, weight_decay=0.1)
    for _ in range(3):
        g1, g2 = torch.randn(10, 3), torch.randn(7)
        opt.zero_grad()
        p1.grad.add_(g1)
        p2.grad.add_(g2)  # views into the flat grad buffer
        opt.step()
        q1.grad, q2.grad = g1.clone(), g2.clone()
        ref.step()
    torch.testing.assert_close(p1.detach(), q1.detach(), atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(p2.detach(), q2.detach(), atol=1e-6, rtol=1e-5)
    assert lr_at(0, 1.0, 10, 100) == pytest.approx(0.1) and lr_at(100, 1.0, 10, 100) == pytest.approx(0.1)


def test_trainer_resume(tmp_path):
    base = dict(model="llama-tiny", method="lora", batch_size=2, seq_len=32, synthetic=True, log_interval=2,
                checkpoint_path=str(tmp_path), lr=1e-2, warmup_steps=0, device="cpu", save_every=2)
    tr = Trainer(TrainConfig(max_steps=4, **base))
    tr.run()
    tr.close()
    assert os.path.exists(tmp_path / "adapter_model.safetensors")
    resume = [f for f in os.listdir(tmp_path) if f.startswith("checkpoint_step")]
    assert resume == ["checkpoint_step2.pt"]
    tr2 = Trainer(TrainConfig(max_steps=6, **base))
    last = tr2.run()
    tr2.close()
    rows = open(tmp_path / "metrics.csv").read().strip().splitlines()
    assert last["step"] == 6 and rows[0].startswith("epoch,step,loss") and rows[-1].split(",")[1] == "6"
    # the first attempt logged step 4 after its last resume checkpoint (step 2); the resumed run logs
    # step 4 again -- the file keeps one row per step
    steps = [int(r.split(",")[1]) for r in rows[1:]]
    assert steps == sorted(set(steps)) and 4 in steps


def test_resume_save_is_durable_and_sweeps_stale_tmp(tmp_path, monkeypatch):
    """The resume file reaches the disk before its rename (the previous resume point is deleted right
    after), and a .tmp a crashed save left behind -- checkpoint-sized -- is removed by the next save."""
    from finetune_controller_amd.models import checkpoint as ckmod

    events = []
    real_fsync, real_replace = os.fsync, os.replace
    monkeypatch.setattr(ckmod.os, "fsync", lambda fd: (events.append("fsync"), real_fsync(fd))[1])
    monkeypatch.setattr(ckmod.os, "replace", lambda a, b: (events.append("replace"), real_replace(a, b))[1])
    (tmp_path / "checkpoint_step1.pt.tmp").write_bytes(b"\0" * 64)  # interrupted save of a previous attempt
    tr = Trainer(TrainConfig(model="llama-tiny", method="lora", batch_size=2, seq_len=32, synthetic=True,
                             checkpoint_path=str(tmp_path), device="cpu", save_every=2, max_steps=3,
                             save_model=False))
    tr.run()
    tr.close()
    assert sorted(f for f in os.listdir(tmp_path) if f.startswith("checkpoint_step")) == ["checkpoint_step2.pt"]
    assert events[:3] == ["fsync", "replace", "fsync"]  # file data, rename, directory entry
    (tmp_path / "checkpoint_step_best.pt").write_bytes(b"")  # a name the trainer never writes
    assert ckpt.latest_resume(str(tmp_path)).endswith("checkpoint_step2.pt")


def test_dataset_formats(tmp_path):
    (tmp_path / "a.jsonl").write_text('{"text": "hello world"}\n{"prompt": "q", "completion": "a"}\n')
    arr = load_token_array(str(tmp_path / "a.jsonl"), vocab=512)
    assert arr.dtype == np.int32 and arr.max() < 512 and len(arr) > 10  # 4 bytes per token while resident
    toks = np.arange(1000, dtype=np.uint16) % 300
    toks.tofile(tmp_path / "t.bin")
    ds = PackedTokenDataset(str(tmp_path / "t.bin"), vocab=512, batch=2, seq_len=16, device="cpu", seed=0)
    x, y = next(ds)
    assert x.shape == (2, 16) and torch.equal(x[:, 1:], y[:, :-1])
    (tmp_path / "c.csv").write_text("Id,SMILES,esol\na,CCO,1.0\nb,CCC,2.0\n")
    assert len(load_token_array(str(tmp_path / "c.csv"), vocab=512)) > 4


def test_text_dataset_edge_cases(tmp_path, monkeypatch):
    """Exports with a byte-order mark, a pretty-printed JSON array, ragged CSV rows, null fields;
    malformed records and a tokenizer larger than the model are refused, not trained on."""
    from finetune_controller_amd.train import data as dmod

    byte_ids = lambda t: [b + 3 for b in t.encode()] + [2]  # noqa: E731  (byte-level fallback + EOS)
    d = tmp_path / "j"
    d.mkdir()
    (d / "a.json").write_bytes(b"\xef\xbb\xbf\n  [\n {\"text\": \"ab\"},\n \"cd\",\n {\"prompt\": null, \"completion\": \"e\"}\n]\n")
    assert load_token_array(str(d / "a.json"), 512).tolist() == byte_ids("ab") + byte_ids("cd") + byte_ids("e")
    (tmp_path / "r.csv").write_text("Id,SMILES\na,CCO\nshort\n\nb,CN\n")
    assert load_token_array(str(tmp_path / "r.csv"), 512).tolist() == byte_ids("CCO") + byte_ids("CN")
    (tmp_path / "bad.jsonl").write_text('{"text": "ok"}\n[1, 2]\n')
    with pytest.raises(ValueError, match="record 1 is a list"):
        load_token_array(str(tmp_path / "bad.jsonl"), 512)
    # batching does not change the token stream (records straddle the batch boundaries)
    rows = [{"prompt": "p%d" % i, "completion": "c" * (i % 7)} if i % 3 else {"text": "t%d" % i} for i in range(50)]
    (tmp_path / "m.jsonl").write_text("\n".join(json.dumps(r) for r in rows))
    whole, wmask = load_tokens_and_mask(str(tmp_path / "m.jsonl"), 512, completion_only=True)
    monkeypatch.setattr(dmod, "TEXT_BATCH", 4)
    parts, pmask = load_tokens_and_mask(str(tmp_path / "m.jsonl"), 512, completion_only=True)
    assert whole.tolist() == parts.tolist() and wmask.tolist() == pmask.tolist()
    # a tokenizer.json of a larger vocabulary than the model's is refused (ids used to be wrapped mod vocab)
    from tokenizers import Tokenizer as HFTok
    from tokenizers.models import WordLevel
    from tokenizers.pre_tokenizers import Whitespace

    vocab = {"[UNK]": 0, "</s>": 1, "hello": 2, "world": 600}
    tk = HFTok(WordLevel(vocab, unk_token="[UNK]"))
    tk.pre_tokenizer = Whitespace()
    t = tmp_path / "t"
    t.mkdir()
    tk.save(str(t / "tokenizer.json"))
    (t / "d.txt").write_text("hello world\nhello\n")
    assert load_token_array(str(t), 1024).tolist() == [2, 600, 1, 2, 1]
    with pytest.raises(ValueError, match="tokenizer ids reach 600"):
        load_token_array(str(t), 512)


@pytest.mark.parametrize("dtype,vocab,ext", [(np.uint16, 512, "bin"), (np.uint32, 100000, "bin"),
                                             (np.int32, 128256, "npy"), (np.uint16, 512, "npy")])
def test_native_token_loader_matches_numpy_path(tmp_path, monkeypatch, dtype, vocab, ext):
    """csrc/runtime token loader (mmap + prefetch threads) yields exactly the numpy path's batches,
    across epoch boundaries, per rank, and after a resume seek -- raw .bin files and .npy files (whose
    header the native loader must skip: reading it as tokens produced ids far past the vocabulary)."""
    pytest.importorskip("finetune_controller_amd._rt")
    toks = (np.arange(5000, dtype=np.int64) * 7919 % vocab).astype(dtype)
    if ext == "npy":
        name = "t.npy"
        np.save(tmp_path / name, toks, allow_pickle=False)
    else:
        name = "t.u32.bin" if dtype == np.uint32 else "t.bin"
        toks.tofile(tmp_path / name)
    for rank in (0, 1):
        monkeypatch.setenv("FTC_NATIVE_LOADER", "1")
        nat = PackedTokenDataset(str(tmp_path / name), vocab=vocab, batch=3, seq_len=32, device="cpu", rank=rank,
                                 world=2, seed=4)
        assert nat._native is not None
        monkeypatch.setenv("FTC_NATIVE_LOADER", "0")
        ref = PackedTokenDataset(str(tmp_path / name), vocab=vocab, batch=3, seq_len=32, device="cpu", rank=rank,
                                 world=2, seed=4)
        assert ref._native is None
        for _ in range(2 * nat.steps_per_epoch + 3):  # crosses two epoch boundaries
            (xa, ya), (xb, yb) = next(nat), next(ref)
            assert torch.equal(xa, xb) and torch.equal(ya, yb)
        st = ref.state()
        nat.load_state(st)
        ref.load_state(st)
        for _ in range(3):
            assert torch.equal(next(nat)[0], next(ref)[0])
        nat._native.close()


def test_negative_int16_token_ids_fail_on_the_host(tmp_path, monkeypatch):
    """A signed int16 file is never read as unsigned by the native loader (-1 would become 65535, a valid
    id of a 128k vocabulary): it takes the numpy path, whose range check rejects the negative id."""
    monkeypatch.setenv("FTC_NATIVE_LOADER", "1")
    toks = (np.arange(4000, dtype=np.int64) % 500).astype(np.int16)
    toks[777] = -1
    np.save(tmp_path / "t.npy", toks, allow_pickle=False)
    ds = PackedTokenDataset(str(tmp_path / "t.npy"), vocab=128256, batch=4, seq_len=64, device="cpu", seed=1)
    assert ds._native is None
    with pytest.raises((ValueError, RuntimeError)):
        for _ in range(2 * ds.steps_per_epoch):
            next(ds)


@pytest.mark.parametrize("native", ["0", "1"])
def test_out_of_vocab_token_ids_fail_on_the_host(tmp_path, monkeypatch, native):
    """A dataset id >= the model's vocabulary (wrong tokenizer) must raise a clear error on the host --
    on the GPU it would make the embedding gather fault the device."""
    if native == "1":
        pytest.importorskip("finetune_controller_amd._rt")
    monkeypatch.setenv("FTC_NATIVE_LOADER", native)
    toks = (np.arange(4000, dtype=np.int64) % 500).astype(np.int32)
    toks[1234] = 700  # one bad id
    np.save(tmp_path / "t.npy", toks, allow_pickle=False)
    ds = PackedTokenDataset(str(tmp_path / "t.npy"), vocab=512, batch=4, seq_len=64, device="cpu", seed=1)
    assert (ds._native is not None) == (native == "1")
    with pytest.raises((ValueError, RuntimeError), match="512"):
        for _ in range(2 * ds.steps_per_epoch):
            next(ds)
    if ds._native is not None:
        ds._native.close()


@pytest.mark.parametrize("native", ["0", "1"])
def test_holdout_windows_never_trained_on(tmp_path, monkeypatch, native):
    """With a held-out split the training order (numpy and native loader) only visits the leading
    windows and EvalWindows only the tail ones."""
    if native == "1":
        pytest.importorskip("finetune_controller_amd._rt")
    monkeypatch.setenv("FTC_NATIVE_LOADER", native)
    S = 16
    np.arange(4000, dtype=np.uint16).tofile(tmp_path / "t.bin")  # window w starts with token w * S
    for rank in (0, 1):
        ds = PackedTokenDataset(str(tmp_path / "t.bin"), vocab=8192, batch=2, seq_len=S, device="cpu", rank=rank,
                                world=2, seed=3, holdout=0.1)
        assert ds.holdout == round(ds.n_windows * 0.1) and ds.n_use + ds.holdout == ds.n_windows
        seen = set()
        for _ in range(3 * ds.steps_per_epoch):
            x, _ = next(ds)
            seen |= {int(v) // S for v in x[:, 0]}
        assert max(seen) < ds.n_use
        ev = [int(v) // S for x, _ in EvalWindows(ds, 3).batches() for v in x[:, 0]]
        assert len(ev) == 6 and all(ds.n_use <= w < ds.n_windows for w in ev)
        if ds._native is not None:
            ds._native.close()


def test_trainer_eval_loss_no_grad_side_effects(tmp_path):
    """Trainer.evaluate: mean held-out loss equal to a direct forward over the tail windows, no
    gradient written (full fine-tuning: the fused CE would otherwise fill lm_head's main_grad), rows in
    metrics.csv."""
    vocab = 512
    (np.arange(6000, dtype=np.int64) * 7919 % vocab).astype(np.uint16).tofile(tmp_path / "t.bin")
    tc = TrainConfig(model="llama-tiny", method="full", batch_size=2, seq_len=32, dataset_path=str(tmp_path / "t.bin"),
                     max_steps=4, log_interval=2, eval_every=2, eval_batches=2, eval_holdout=0.05,
                     checkpoint_path=str(tmp_path / "out"), resume=False, device="cpu", lr=1e-3, warmup_steps=0,
                     save_model=False)
    tr = Trainer(tc)
    tr.train_step(1e-3)
    g0 = tr.opt.grad_flat.detach().clone()
    ev = tr.evaluate()
    assert torch.equal(tr.opt.grad_flat, g0) and tr.model.training
    ds = tr.data()
    ref = []
    with torch.no_grad():
        for x, y in EvalWindows(ds, 2).batches():
            ref.append(float(tr.model(x, y)))
    assert ev == pytest.approx(sum(ref) / len(ref), rel=1e-5)
    last = tr.run()
    tr.close()
    rows = read_metrics_csv(str(tmp_path / "out" / "metrics.csv"))
    evals = [r for r in rows if r["eval_loss"]]
    assert [r["step"] for r in evals] == [2, 4] and all(0 < r["eval_loss"] < 20 for r in evals)
    assert last["eval_loss"] == evals[-1]["eval_loss"]


def test_trainer_eval_synthetic(tmp_path):
    tr = Trainer(TrainConfig(model="llama-tiny", method="lora", batch_size=2, seq_len=16, synthetic=True,
                             max_steps=1, eval_batches=3, checkpoint_path=str(tmp_path), resume=False, device="cpu",
                             save_model=False))
    a, b = tr.evaluate(), tr.evaluate()
    tr.close()
    assert a == b and a == pytest.approx(np.log(512), rel=0.1)


def test_attached_dataset_missing_fails_instead_of_synthetic(tmp_path, monkeypatch):
    """Without a dataset a dataset-optional spec trains on synthetic tokens; with FTC_DATASET_EXPECTED=1
    (the manifest sets it when the job has a dataset) an empty mount -- a failed download -- must fail
    the worker rather than 'complete' on random tokens."""
    empty = tmp_path / "dataset"
    empty.mkdir()

    def trainer():
        return Trainer(TrainConfig(model="llama-tiny", method="lora", batch_size=2, seq_len=16,
                                   dataset_path=str(empty), max_steps=1, checkpoint_path=str(tmp_path / "ck"),
                                   resume=False, device="cpu", save_model=False))

    monkeypatch.delenv("FTC_DATASET_EXPECTED", raising=False)
    tr = trainer()
    assert type(tr.data()).__name__ == "SyntheticTokens"
    tr.close()
    monkeypatch.setenv("FTC_DATASET_EXPECTED", "1")
    tr = trainer()
    with pytest.raises(FileNotFoundError, match="missing or empty"):
        tr.data()
    tr.close()


def _hold_until_released(tmp, port, timeout=120.0):
    """Keep a spawned rank alive until the parent has read its queued tensors: torch shares them by
    file descriptor through the sender, so a sender that exits first resets the parent's read."""
    import time

    t0 = time.time()
    while not os.path.exists(os.path.join(tmp, f"release_{port}")) and time.time() - t0 < timeout:
        time.sleep(0.05)


def _release(tmp, port):
    open(os.path.join(tmp, f"release_{port}"), "w").close()


def _ddp_worker(rank, world, port, tmp, q):
    # file rendezvous in the test dir: a picked-then-released TCP port can be taken by a parallel test
    os.environ["FTC_INIT_METHOD"] = f"file://{tmp}/rdv_{port}"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    tc = TrainConfig(model="llama-tiny", method="lora", batch_size=2, seq_len=16, synthetic=True, max_steps=1,
                     checkpoint_path=tmp, resume=False, device="cpu", lr=0.0, bucket_mb=0.01, max_grad_norm=0.0,
                     save_model=False)
    tr = Trainer(tc)
    tr.train_step(0.0)
    q.put((rank, tr.opt.grad_flat.detach().clone(), [b for b in tr.ddp.buckets]))
    tr.close()
    _hold_until_released(tmp, port)


def test_ddp_gloo_two_ranks_matches_single_process(tmp_path):
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, b)) for r, g, b in (q.get(timeout=120) for _ in range(2)))
    _release(str(tmp_path), port)
    for p in procs:
        p.join(timeout=60)
    g0, buckets = res[0]
    g1, _ = res[1]
    assert len(buckets) > 1  # several buckets were launched during backward
    torch.testing.assert_close(g0, g1)  # all-reduced (summed) gradients identical on both ranks
    # single-process reference: sum of the two ranks' local gradients (rank seeds differ in data only)
    grads = []
    for rank in range(2):
        tc = TrainConfig(model="llama-tiny", method="lora", batch_size=2, seq_len=16, synthetic=True, max_steps=1,
                         checkpoint_path=str(tmp_path), resume=False, device="cpu", lr=0.0, max_grad_norm=0.0,
                         save_model=False, seed=1)
        tr = Trainer(tc)
        tr._data = None
        from finetune_controller_amd.train.data import SyntheticTokens

        tr._data = SyntheticTokens(tr.cfg.vocab_size, 2, 16, "cpu", seed=1 + rank)
        tr.steps_per_epoch = 100
        tr.train_step(0.0)
        grads.append(tr.opt.grad_flat.detach().clone())
        tr.close()
    torch.testing.assert_close(g0, grads[0] + grads[1], atol=1e-5, rtol=1e-4)


def test_lora_dropout_matches_autograd_reference():
    """PEFT-style LoRA dropout (adapter input only): output and all grads against autograd on the same
    mask (same RNG draw)."""
    torch.manual_seed(0)
    x = torch.randn(7, 16, requires_grad=True)
    W = torch.randn(12, 16)
    A = torch.randn(4, 16, requires_grad=True)
    B = torch.randn(12, 4, requires_grad=True)
    p = 0.3
    torch.manual_seed(123)
    y = ops.lora_linear(x, W, A, B, 0.5, dropout=p)
    torch.manual_seed(123)
    mask = torch.rand(7, 16) >= p
    x2, A2, B2 = (t.detach().clone().requires_grad_(True) for t in (x, A, B))
    ref = x2 @ W.t() + 0.5 * ((x2 * mask / (1 - p)) @ A2.t()) @ B2.t()
    torch.testing.assert_close(y, ref)
    g = torch.randn_like(y)
    y.backward(g)
    ref.backward(g)
    for a_, b_ in ((x.grad, x2.grad), (A.grad, A2.grad), (B.grad, B2.grad)):
        torch.testing.assert_close(a_, b_)


def _zero_worker(rank, world, port, tmp, zero, q):
    # file rendezvous in the test dir: a picked-then-released TCP port can be taken by a parallel test
    os.environ["FTC_INIT_METHOD"] = f"file://{tmp}/rdv_{port}"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    tc = TrainConfig(model="llama-tiny", method="lora", batch_size=2, seq_len=16, synthetic=True, max_steps=3,
                     checkpoint_path=tmp, resume=False, device="cpu", lr=1e-2, bucket_mb=0.01, max_grad_norm=0.5,
                     save_model=False, zero_stage=zero, weight_decay=0.1)
    tr = Trainer(tc)
    for _ in range(3):
        tr.train_step(1e-2)
    sd = tr.opt.state_dict()  # collective under ZeRO-1
    out = {"param": tr.opt.param_flat.detach().clone(), "gn": tr.opt.grad_norm(),
           "exp_avg": sd["exp_avg"].detach().cpu().clone(), "n_buckets": len(tr.ddp.buckets),
           "sharded": hasattr(tr.opt, "grad_shard")}
    if zero:
        # resume path: a fresh sharded optimizer takes the gathered full-layout state back
        from finetune_controller_amd.train.optim import ShardedFlatAdamW

        opt2 = ShardedFlatAdamW([p for p in tr.model.parameters() if p.requires_grad], world, rank,
                                bucket_elems=tr.opt.bucket_elems, lr=1e-2)
        opt2.load_state_dict(sd)
        out["reload_ok"] = bool(torch.equal(opt2.exp_avg, tr.opt.exp_avg) and torch.equal(opt2.master, tr.opt.master))
    q.put((rank, out))
    tr.close()
    _hold_until_released(tmp, port)


@pytest.mark.parametrize("world", [2, 3])
def test_zero1_sharded_optimizer_matches_ddp(tmp_path, world):
    """ZeRO-1 (reduce-scatter grads, sharded AdamW, in-place all-gather) over gloo reproduces the
    all-reduce DDP trajectory: parameters after 3 clipped AdamW steps, grad norm, gathered moments."""
    import socket

    runs = {}
    for zero in (0, 1):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_zero_worker, args=(r, world, port, str(tmp_path), zero, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = dict(q.get(timeout=180) for _ in range(world))
        _release(str(tmp_path), port)
        for p in procs:
            p.join(timeout=60)
        runs[zero] = res
    for r in range(world):
        assert runs[1][r]["sharded"] and not runs[0][r]["sharded"]
        torch.testing.assert_close(runs[1][r]["param"], runs[1][0]["param"], atol=0, rtol=0)
        assert runs[1][r]["reload_ok"]
    assert runs[1][0]["n_buckets"] > 1
    # same trajectory as DDP (layouts differ only by bucket padding: compare the live parameters)
    p0, p1 = runs[0][0]["param"], runs[1][0]["param"]

    assert abs(runs[0][0]["gn"] - runs[1][0]["gn"]) < 1e-4 * max(1.0, runs[0][0]["gn"])
    live0 = p0[p0 != 0]
    live1 = p1[p1 != 0]
    # reduction orders differ (reduce-scatter vs all-reduce); AdamW steps are lr = 1e-2 per element
    torch.testing.assert_close(live1, live0, atol=1e-4, rtol=1e-3)


@pytest.mark.parametrize("name", ["llama3.1-8b", "llama3.2-1b", "llama3.2-3b", "llama3-70b", "mistral-7b-v0.3"])
def test_llama_family_presets(name):
    """Llama-trunk presets: public parameter counts, HF config round trip (rope scaling, tied
    embeddings), and a LoRA step of a width-reduced copy on the CPU reference path."""
    import dataclasses

    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import ModelConfig, get_config

    expect = {"llama3.1-8b": 8.03, "llama3.2-1b": 1.24, "llama3.2-3b": 3.21, "llama3-70b": 70.55,
              "mistral-7b-v0.3": 7.25}
    cfg = get_config(name)
    assert abs(cfg.num_params() / 1e9 - expect[name]) < 0.01
    back = ModelConfig.from_hf_config(cfg.to_hf_config(), name=name)
    assert (back.rope_scaling, back.tie_embeddings, back.n_kv_heads, back.rope_theta) == \
        (cfg.rope_scaling, cfg.tie_embeddings, cfg.n_kv_heads, cfg.rope_theta)
    small = dataclasses.replace(cfg, vocab_size=512, dim=cfg.head_dim * 4, n_layers=1, n_heads=4,
                                n_kv_heads=4 // max(1, cfg.n_heads // cfg.n_kv_heads) or 1, ffn_dim=256,
                                max_seq_len=64)
    torch.manual_seed(0)
    m = build_model(small, LoRAConfig(r=4, alpha=8), dtype=torch.float32)
    m.init_weights(seed=1)
    m.freeze_base()
    ids = torch.randint(0, 512, (2, 32))
    loss = m(ids, torch.roll(ids, -1, 1))
    loss.backward()
    assert torch.isfinite(loss) and all(p.grad is not None for p in m.parameters() if p.requires_grad)


def test_rslora_scale_and_adapter_config(tmp_path):
    from finetune_controller_amd.models import LoRAConfig

    lc = LoRAConfig(r=16, alpha=32, use_rslora=True)
    assert lc.scale == pytest.approx(32 / 4.0) and LoRAConfig(r=16, alpha=32).scale == 2.0
    tr = Trainer(TrainConfig(model="llama-tiny", method="lora", use_rslora=True, lora_r=8, lora_alpha=16,
                             batch_size=1, seq_len=16, synthetic=True, max_steps=1, checkpoint_path=str(tmp_path),
                             resume=False, device="cpu"))
    assert all(p.scale == pytest.approx(16 / 8 ** 0.5) for layer in tr.model.layers for p in layer.lora.values())
    tr.run()
    tr.close()
    assert json.load(open(tmp_path / "adapter_config.json"))["use_rslora"] is True


def test_dw_split_choices_on_llama3_8b_shapes():
    """Split-K weight gradients (ops.linear.dw_splits, FTC_DW_SPLIT=auto): only the wave-quantised wide-input
    shape splits (down 896 tiles -> 2 x); qkv (measured faster unsplit), whole-wave and huge grids do not."""
    from finetune_controller_amd.ops.linear import dw_splits

    T = 16384
    assert dw_splits(6144, 4096, T, "auto") == 1   # qkv
    assert dw_splits(4096, 14336, T, "auto") == 2  # down
    assert dw_splits(4096, 4096, T, "auto") == 1   # o: one whole wave
    assert dw_splits(28672, 4096, T, "auto") == 1  # gate | up: seven whole waves
    assert dw_splits(6144, 4096, T, "0") == 1
    assert dw_splits(6144, 4096, T, "4") == 4
    assert dw_splits(6144, 4096, 192, "4") == 1    # slices must stay multiples of 64 tokens
