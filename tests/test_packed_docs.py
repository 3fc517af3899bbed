"""Packed documents (several EOS-separated documents per row): segment bounds, document-masked
attention, per-document positions, and the trainer's label masking -- CPU (torch path)."""
import math

import pytest
import torch

from finetune_controller_amd import ops
from finetune_controller_amd.models import build_model
from finetune_controller_amd.models.config import get_config
from finetune_controller_amd.ops.attention import attention_reference, segments_from_eos
from finetune_controller_amd.train.trainer import Trainer, TrainConfig


def test_segments_from_eos():
    ids = torch.tensor([[5, 2, 7, 8, 2, 9], [1, 1, 1, 1, 1, 2]])
    s = segments_from_eos(ids, 2)
    assert s.doc_start.view(2, 6).tolist() == [[0, 0, 2, 2, 2, 5], [0] * 6]
    assert s.doc_end.view(2, 6).tolist() == [[2, 2, 5, 5, 5, 6], [6] * 6]
    assert s.positions.view(2, 6).tolist() == [[0, 1, 0, 1, 2, 0], [0, 1, 2, 3, 4, 5]]
    assert s.doc_start.dtype == torch.int32 and s.doc_start.is_contiguous()


def _docs_batch(lens, vocab, eos, gen):
    """One row of EOS-terminated documents of the given lengths (EOS included)."""
    parts = []
    for n in lens:
        t = torch.randint(3, vocab, (n,), generator=gen)
        t[-1] = eos
        parts.append(t)
    return torch.cat(parts)


def test_document_masked_attention_matches_separate_documents():
    torch.manual_seed(0)
    B, S, H, KV, D = 1, 48, 4, 2, 16
    lens = [10, 20, 18]
    ids = torch.zeros(1, S, dtype=torch.long)
    ends = torch.tensor(lens).cumsum(0)
    ids[0, ends - 1] = 2
    seg = segments_from_eos(ids, 2)
    qkv = torch.randn(B * S, (H + 2 * KV) * D)
    out = ops.attention_packed(qkv, B, S, H, KV, D, docs=seg)
    ref = attention_reference(qkv, B, S, H, KV, D, docs=seg)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
    lo = 0
    for n in lens:
        alone = attention_reference(qkv[lo:lo + n], 1, n, H, KV, D)
        torch.testing.assert_close(out[lo:lo + n], alone, atol=1e-5, rtol=1e-5)
        lo += n


@pytest.mark.parametrize("preset", ["llama-tiny", "gpt2-tiny"])
def test_packed_model_equals_documents_run_alone(preset):
    """Logits of a packed row (segments: masked attention + restarted positions) equal the logits of
    each document run as its own sequence."""
    cfg = get_config(preset)
    torch.manual_seed(0)
    m = build_model(cfg, None, device="cpu", dtype=torch.float32)
    m.init_weights(seed=3)
    m.eval()
    g = torch.Generator().manual_seed(1)
    lens = [7, 13, 12]
    row = _docs_batch(lens, cfg.vocab_size, 2, g)[None]
    seg = segments_from_eos(row, 2)
    with torch.no_grad():
        packed = m(row, segments=seg)
        lo = 0
        for n in lens:
            alone = m(row[:, lo:lo + n])
            torch.testing.assert_close(packed[lo:lo + n], alone.reshape(n, -1), atol=2e-4, rtol=2e-4)
            lo += n


def test_trainer_pack_documents_masks_boundary_labels(tmp_path):
    import numpy as np

    g = torch.Generator().manual_seed(2)
    toks = torch.cat([_docs_batch([int(n)], 512, 2, g) for n in torch.randint(5, 40, (200,), generator=g)])
    toks.numpy().astype(np.uint16).tofile(tmp_path / "t.bin")
    tr = Trainer(TrainConfig(model="llama-tiny", method="lora", batch_size=2, seq_len=64,
                             dataset_path=str(tmp_path / "t.bin"), max_steps=3, log_interval=1, pack_documents=True,
                             eos_id=2, checkpoint_path=str(tmp_path / "out"), resume=False, device="cpu",
                             save_model=False, warmup_steps=0, lr=1e-3))
    data = tr.data()
    x, y = next(data)
    x2, y2, seg, n_valid = tr._batch(x, y, data)
    n_eos = int((x == 2).sum())
    assert n_eos > 0 and n_valid == x.numel() - n_eos == data.last_n_valid
    assert bool((y2[x == 2] == -100).all()) and bool((y2[x != 2] != -100).all())
    keep = x[:, :-1] != 2
    assert bool((y2[:, :-1][keep] == x[:, 1:][keep]).all())  # kept labels are the next inputs
    assert seg.positions.max() < 64
    last = tr.run()
    tr.close()
    assert math.isfinite(last["loss"])


def test_completion_only_masks_prompt_labels(tmp_path):
    import json

    from finetune_controller_amd.train.data import PackedTokenDataset, load_tokens_and_mask

    rows = [{"prompt": "Q: what is %d+%d? A:" % (i, i), "completion": " %d" % (2 * i)} for i in range(60)]
    (tmp_path / "d.jsonl").write_text("\n".join(json.dumps(r) for r in rows))
    ids, mask = load_tokens_and_mask(str(tmp_path / "d.jsonl"), 512, completion_only=True)
    assert mask is not None and len(mask) == len(ids) and 0 < mask.sum() < len(mask)
    # byte-level fallback: the first record's prompt bytes are masked, its completion + EOS are not
    n_p = len("Q: what is 0+0? A:".encode())
    assert mask[:n_p].sum() == 0 and mask[n_p:n_p + 3].tolist() == [1, 1, 1] and ids[n_p + 2] == 2
    assert load_tokens_and_mask(str(tmp_path / "d.jsonl"), 512)[1] is None
    ds = PackedTokenDataset(str(tmp_path / "d.jsonl"), 512, batch=2, seq_len=32, device="cpu", completion_only=True)
    x, y = next(ds)
    assert ds._native is None and ds.last_n_valid == int((y != -100).sum()) < y.numel()
    # a label is kept iff the token it predicts is a completion token
    S = 32
    j = int(ds.order[0])
    keep = torch.from_numpy(mask[j * S + 1: j * S + S + 1].astype(bool))
    assert torch.equal(y[0] != -100, keep)
    tr = Trainer(TrainConfig(model="llama-tiny", method="lora", batch_size=2, seq_len=32,
                             dataset_path=str(tmp_path / "d.jsonl"), max_steps=2, completion_only=True,
                             checkpoint_path=str(tmp_path / "out"), resume=False, device="cpu", save_model=False,
                             warmup_steps=0))
    assert math.isfinite(tr.run()["loss"])
    tr.close()


def test_native_loader_label_masking_matches_numpy(tmp_path, monkeypatch):
    import numpy as np

    pytest.importorskip("finetune_controller_amd._rt")
    from finetune_controller_amd.train.data import PackedTokenDataset

    toks = (np.arange(6000) * 7919 % 300).astype(np.uint16)
    toks[::37] = 2
    toks.tofile(tmp_path / "t.bin")
    out = {}
    for native in ("1", "0"):
        monkeypatch.setenv("FTC_NATIVE_LOADER", native)
        ds = PackedTokenDataset(str(tmp_path / "t.bin"), 512, batch=3, seq_len=64, device="cpu", seed=5, eos_id=2)
        assert (ds._native is not None) == (native == "1")
        out[native] = [(*next(ds), ds.last_n_valid) for _ in range(5)]
        if ds._native is not None:
            ds._native.close()
    for (xa, ya, na), (xb, yb, nb) in zip(out["1"], out["0"]):
        assert torch.equal(xa, xb) and torch.equal(ya, yb) and na == nb and bool((ya[xa == 2] == -100).all())
