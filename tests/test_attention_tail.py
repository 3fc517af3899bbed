"""Tail padding for sequence lengths that are not a multiple of the flash kernels' 256-row tile
(ops/attention.py:_FlashPaddedTail).

On the CPU the HIP kernels are replaced by an exact torch implementation with the kernels' calling
convention (``flash_fwd`` -> (o, lse), ``flash_bwd`` writing dq/dk/dv in place, per-token
``doc_start`` / ``doc_end`` bounds), so what is tested here is the padding wrapper itself: forward
and gradients against the unpadded fp64 reference, with windows and packed documents.  The same
shapes against the real kernels are in tests/test_kernels_gpu.py (``test_flash_tail_lengths``).
"""
import math

import pytest
import torch

from finetune_controller_amd.ops import attention as A


class _TorchFlash:
    """The kernels' contract in torch (fp64 math)."""

    @staticmethod
    def _mask(B, S, causal, window, doc_start, device, kv_valid=-1):
        i = torch.arange(S, device=device)
        allowed = torch.ones(S, S, dtype=torch.bool, device=device)
        if 0 < kv_valid < S:  # keys past the valid length are masked for every query
            allowed &= i[None, :] < kv_valid
        if causal:
            allowed &= i[None, :] <= i[:, None]
        if window:
            allowed &= (i[:, None] - i[None, :]) < window
        allowed = allowed.expand(B, 1, S, S)
        if doc_start is not None:
            ds = doc_start.view(B, S).long()
            allowed = allowed & (i[None, None, None, :] >= ds[:, None, :, None])
        return allowed

    def _fwd(self, q, k, v, B, S, H, KV, D, scale, causal, window, doc_start, kv_valid=-1):
        qh = q.double().reshape(B, S, H, D).transpose(1, 2)
        kh = k.double().reshape(B, S, KV, D).transpose(1, 2).repeat_interleave(H // KV, 1)
        vh = v.double().reshape(B, S, KV, D).transpose(1, 2).repeat_interleave(H // KV, 1)
        s = (qh @ kh.transpose(-1, -2)) * scale
        s = s.masked_fill(~self._mask(B, S, causal, window, doc_start, q.device, kv_valid), float("-inf"))
        lse = torch.logsumexp(s, -1)
        o = (s - lse[..., None]).exp() @ vh
        return o.transpose(1, 2).reshape(B * S, H * D), lse

    def flash_fwd(self, q, k, v, B, S, H, KV, D, scale, causal, window, out_pad, doc_start, kv_valid=-1):
        o, lse = self._fwd(q, k, v, B, S, H, KV, D, scale, causal, window, doc_start, kv_valid)
        buf = torch.empty(B * S, H * D + out_pad, dtype=q.dtype)[:, :H * D]
        buf.copy_(o)
        return buf, lse.float()

    def flash_bwd(self, q, k, v, o, do, lse, dq, dk, dv, B, S, H, KV, D, scale, causal, window, doc_start, doc_end,
                  kv_valid=-1):
        with torch.enable_grad():  # called from inside autograd's backward
            qq, kk, vv = (t.detach().double().requires_grad_(True) for t in (q, k, v))
            out, _ = self._fwd(qq, kk, vv, B, S, H, KV, D, scale, causal, window, doc_start, kv_valid)
            gq, gk, gv = torch.autograd.grad(out, (qq, kk, vv), do.double())
        dq.copy_(gq)
        dk.copy_(gk)
        dv.copy_(gv)


@pytest.mark.parametrize("S,window,docs,causal,D", [(300, 0, False, True, 64), (1000, 0, False, True, 64),
                                                    (300, 64, False, True, 64), (520, 0, True, True, 64),
                                                    (300, 0, False, False, 64), (1000, 0, False, False, 64),
                                                    (256, 0, False, True, 96), (300, 0, False, True, 80),
                                                    (520, 0, True, True, 96), (300, 0, False, False, 112),
                                                    (256, 40, False, True, 32)])
def test_padded_tail_matches_reference(monkeypatch, S, window, docs, causal, D):
    """Tail rows (S off the tile) and/or zero head columns (D not a kernel head_dim) are exact."""
    seen = []

    class _Rec(_TorchFlash):
        def flash_fwd(self, q, k, v, B, S, H, KV, D, *a):
            seen.append((S, D))
            return super().flash_fwd(q, k, v, B, S, H, KV, D, *a)

    monkeypatch.setattr(A, "ext", lambda: _Rec())
    B, H, KV = 2, 4, 2
    torch.manual_seed(0)
    W = (H + 2 * KV) * D
    qkv = torch.randn(B * S, W, dtype=torch.float64)
    seg = None
    if docs:
        ids = torch.randint(3, 50, (B, S))
        ids[0, 100] = ids[0, 333] = ids[1, 17] = 2  # documents end at EOS
        seg = A.segments_from_eos(ids, 2)
    scale = 1 / math.sqrt(D)
    x1 = qkv.clone().requires_grad_(True)
    out_pad, grad_pad = 64, 32
    o = A._FlashPaddedTail.apply(x1, B, S, H, KV, D, window, scale, out_pad, grad_pad, seg, causal)
    assert o.shape == (B * S, H * D) and o.stride(0) == H * D + out_pad  # spare columns for the LoRA GEMM
    x2 = qkv.clone().requires_grad_(True)
    ref = A.attention_reference(x2, B, S, H, KV, D, causal, window, scale, seg)
    assert torch.allclose(o, ref.double(), atol=2e-5, rtol=1e-4)  # the reference computes in fp32
    g = torch.randn_like(ref)
    o.backward(g.double())
    ref.backward(g)
    assert torch.allclose(x1.grad, x2.grad, atol=2e-4, rtol=1e-3)
    assert seen == [(-(-S // 256) * 256, A.kernel_head_dim(D))]  # the kernels only ever see their own shapes


def test_flash_usable_policy():
    assert A.flash_supported(128, 4096) and not A.flash_supported(128, 4000)
    assert A.flash_usable(128, 4000, causal=True) and A.flash_usable(64, 77, causal=True)
    assert A.flash_usable(128, 4000, causal=False)  # non-causal: the kernels mask the pad keys (kv_valid)
    assert A.flash_usable(96, 4096, causal=True) and A.flash_usable(80, 1000, causal=False)  # zero-padded heads
    assert not A.flash_supported(96, 4096) and not A.flash_usable(256, 4096, causal=True)
    assert A.kernel_head_dim(32) == 64 and A.kernel_head_dim(96) == 128


@pytest.mark.parametrize("preset,S,docs", [("llama-tiny", 200, False), ("mistral-tiny", 300, False),
                                           ("llama-tiny", 200, True), ("gpt2-tiny", 100, False)])
def test_model_level_tile_padding_is_exact(monkeypatch, preset, S, docs):
    """The GPU path right-pads whole batches to the 256-row tile (ops.attention.model_tile_len): the
    loss, its gradients and the logits must equal the unpadded model's."""
    from finetune_controller_amd import ops
    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import get_config

    cfg = get_config(preset)
    torch.manual_seed(0)
    B = 2
    ids = torch.randint(3, cfg.vocab_size, (B, S))
    if docs:
        ids[0, 50] = ids[1, 120] = 2
    labels = torch.roll(ids, -1, 1)
    labels[:, -1] = -100

    def run(pad: bool):
        torch.manual_seed(1)  # adapters draw from the global RNG
        m = build_model(cfg, LoRAConfig(r=4, alpha=8), device="cpu", dtype=torch.float32)
        m.init_weights(seed=5)
        for layer in getattr(m, "layers", []):
            for pair in layer.lora.values():
                torch.nn.init.normal_(pair.B, std=0.05)
        if pad:
            monkeypatch.setattr(ops, "model_tile_len", lambda S_, *a: -(-S_ // 256) * 256)
        else:
            monkeypatch.setattr(ops, "model_tile_len", lambda S_, *a: S_)
        seg = A.segments_from_eos(ids, 2) if docs else None
        loss = m(ids, labels, n_valid=int((labels != -100).sum()), segments=seg)
        loss.backward()
        grads = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        with torch.no_grad():
            logits = m(ids, segments=seg)
        return loss.detach().item(), grads, logits

    l0, g0, z0 = run(False)
    l1, g1, z1 = run(True)
    assert abs(l0 - l1) < 1e-5 and z0.shape == z1.shape == (B * S, cfg.vocab_size)
    assert torch.allclose(z0, z1, atol=1e-4, rtol=1e-4)
    assert g0.keys() == g1.keys() and all(torch.allclose(g0[k], g1[k], atol=1e-5, rtol=1e-4) for k in g0)
