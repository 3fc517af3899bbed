"""Numerics of every gfx950 HIP kernel against a plain PyTorch fp32 reference of the same op.

Run on an MI355X: ``python -m pytest tests -m gpu``.  These tests import the in-tree extension
directly (``finetune_controller_amd._C``) and fail -- not skip -- when it is missing on a GPU box.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def C():
    import finetune_controller_amd._C as C  # must load: native code is the point of these tests

    return C


def bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("rows,d", [(257, 4096), (64, 768), (33, 128), (8, 8192), (4096, 4096)])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm_fwd_bwd(C, rows, d, with_res):
    torch.manual_seed(0)
    x = bf(torch.randn(rows, d, device=DEV))
    r = bf(torch.randn(rows, d, device=DEV)) if with_res else None
    w = bf(torch.rand(d, device=DEV) + 0.5)
    y, rstd, h = C.rmsnorm_fwd(x, r, w, 1e-5)
    href = (x.float() + r.float()) if with_res else x.float()
    href_b = bf(href).float()
    ref = href_b * torch.rsqrt(href_b.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    if with_res:
        torch.testing.assert_close(h.float(), href_b, atol=0, rtol=0)
    # backward vs autograd in fp32
    dy = bf(torch.randn(rows, d, device=DEV))
    dres = bf(torch.randn(rows, d, device=DEV))
    hv = href_b.clone().requires_grad_(True)
    wv = w.float().clone().requires_grad_(True)
    out = hv * torch.rsqrt(hv.pow(2).mean(-1, keepdim=True) + 1e-5) * wv
    out.backward(dy.float())
    dx, dw = C.rmsnorm_bwd(dy, h if with_res else x, w, rstd, dres, True)
    torch.testing.assert_close(dx.float(), hv.grad + dres.float(), atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(dw, wv.grad, atol=5e-2 * math.sqrt(rows), rtol=2e-2)
    # frozen-weight backward (two waves per row kernel), with and without the residual gradient
    dx2 = C.rmsnorm_bwd(dy, h if with_res else x, w, rstd, dres, False)[0]
    torch.testing.assert_close(dx2.float(), hv.grad + dres.float(), atol=3e-2, rtol=3e-2)
    dx3 = C.rmsnorm_bwd(dy, h if with_res else x, w, rstd, None, False)[0]
    torch.testing.assert_close(dx3.float(), hv.grad, atol=3e-2, rtol=3e-2)


def test_rope_roundtrip_and_reference(C):
    from finetune_controller_amd.ops.rope import RotaryTable, _rope_ref

    torch.manual_seed(0)
    H, KV, D, B, S = 8, 2, 128, 2, 64
    tab = RotaryTable(D, 256, 500000.0)
    cos, sin = tab.get(DEV)
    qkv = bf(torch.randn(B * S, (H + 2 * KV) * D, device=DEV))
    ref = _rope_ref(qkv, cos, sin, H + KV, D, S, None, False)
    out = qkv.clone()
    C.rope_(out, cos, sin, None, H + KV, D, S, False)
    torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)
    # v untouched, inverse restores
    assert torch.equal(out[:, (H + KV) * D:], qkv[:, (H + KV) * D:])
    C.rope_(out, cos, sin, None, H + KV, D, S, True)
    torch.testing.assert_close(out.float(), qkv.float(), atol=3e-2, rtol=3e-2)


def test_swiglu(C):
    torch.manual_seed(0)
    gu = bf(torch.randn(300, 2 * 1024, device=DEV))
    a = C.swiglu_fwd(gu)
    g, u = gu.float().chunk(2, -1)
    torch.testing.assert_close(a.float(), torch.nn.functional.silu(g) * u, atol=2e-2, rtol=2e-2)
    da = bf(torch.randn(300, 1024, device=DEV))
    gv = gu.float().clone().requires_grad_(True)
    gg, uu = gv.chunk(2, -1)
    (torch.nn.functional.silu(gg) * uu).backward(da.float())
    dgu = C.swiglu_bwd(da, gu)
    torch.testing.assert_close(dgu.float(), gv.grad, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("rows,F,R,pad,split", [(200, 384, 16, 64, False), (4096, 1024, 40, 64, False),
                                                 (33, 128, 64, 64, False), (16, 256, 8, 16, False),
                                                 (300, 512, 32, 64, True), (77, 640, 64, 64, True)])
def test_swiglu_lora_tail(C, rows, F, R, pad, split):
    """swiglu_{fwd,bwd}_lora (csrc/kernels/swiglu_lora.hip): the SwiGLU result plus its rank-R product
    in the tail columns of the padded buffer, against fp32 products of the stored bf16 values."""
    torch.manual_seed(0)
    nct = -(-R // 16)
    gu = bf(torch.randn(rows, 2 * F, device=DEV))
    # forward: tail = h (sA)^T with sA the rows of a padded [pad, F (+ extra cols)] operand view
    big = torch.zeros(pad + 3, F + 24, device=DEV, dtype=torch.bfloat16)
    big[:R, :F] = bf(torch.randn(R, F, device=DEV) * 0.1)
    am = big[:pad, :F]
    a = C.swiglu_fwd_lora(gu, pad, am, nct)
    assert a.shape == (rows, F) and a.stride(0) == F + pad
    g, u = gu.float().chunk(2, -1)
    torch.testing.assert_close(a.float(), torch.nn.functional.silu(g) * u, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(a, C.swiglu_fwd(gu), atol=0, rtol=0)  # bit-identical to the plain kernel
    full = a.as_strided((rows, F + pad), (F + pad, 1))
    tail = full[:, F:].float()
    ref = a.float() @ am[:R].float().t()
    torch.testing.assert_close(tail[:, :R], ref, atol=2e-2 * ref.abs().max().item() + 1e-3, rtol=2e-2)
    assert torch.count_nonzero(tail[:, R:]) == 0
    # backward: tail = dgu B with B^T [pad, 2F]
    da = bf(torch.randn(rows, F, device=DEV))
    bt = torch.zeros(pad, 2 * F, device=DEV, dtype=torch.bfloat16)
    bt[:R] = bf(torch.randn(R, 2 * F, device=DEV) * 0.1)
    if split:  # block-diagonal B: gate rows feed tail columns [0, R/2), up rows [R/2, R)
        bt[:R // 2, F:] = 0
        bt[R // 2:R, :F] = 0
    dgu = C.swiglu_bwd_lora(da, gu, pad, bt, nct, split)
    assert dgu.shape == (rows, 2 * F) and dgu.stride(0) == 2 * F + pad
    torch.testing.assert_close(dgu, C.swiglu_bwd(da, gu), atol=0, rtol=0)
    fullb = dgu.as_strided((rows, 2 * F + pad), (2 * F + pad, 1))
    tailb = fullb[:, 2 * F:].float()
    refb = dgu.float() @ bt[:R].float().t()
    torch.testing.assert_close(tailb[:, :R], refb, atol=2e-2 * refb.abs().max().item() + 1e-3, rtol=2e-2)
    assert torch.count_nonzero(tailb[:, R:]) == 0


@pytest.mark.parametrize("T,F", [(1000, 1024), (4096, 512), (77, 512)])
def test_swiglu_bwd_wgrad(C, T, F):
    """swiglu_bwd_wgrad (csrc/kernels/swiglu_lora.hip): dgu, its row tail dgu B and the LoRA weight
    gradients dB_gu += dgu^T xa (block-diagonal gate|up) and dA_down += s dyb^T h in one pass, against
    fp32 products of the stored bf16 values (h = the forward SwiGLU output)."""
    torch.manual_seed(0)
    pad = 64
    gu = bf(torch.randn(T, 2 * F, device=DEV))
    da = bf(torch.randn(T, F, device=DEV))
    bt = torch.zeros(pad, 2 * F, device=DEV, dtype=torch.bfloat16)
    bt[:16, :F] = bf(torch.randn(16, F, device=DEV) * 0.1)
    bt[16:32, F:] = bf(torch.randn(16, F, device=DEV) * 0.1)
    xbuf = bf(torch.randn(T, 104, device=DEV))
    xa = xbuf[:, 40:72]
    ybuf = bf(torch.randn(T, 40, device=DEV))
    dyb = ybuf[:, 8:24]
    mgB = torch.zeros(2 * F, 32, device=DEV, dtype=torch.bfloat16)
    mgB[:F, :16] = bf(torch.randn(F, 16, device=DEV))
    mgB[F:, 16:] = bf(torch.randn(F, 16, device=DEV))
    mgA = bf(torch.randn(16, F, device=DEV))
    mgB0, mgA0 = mgB.float().clone(), mgA.float().clone()
    dgu = C.swiglu_bwd_wgrad(da, gu, pad, bt, xa, dyb, mgB, mgA, 1.0, 0.5)
    assert dgu.shape == (T, 2 * F) and dgu.stride(0) == 2 * F + pad
    torch.testing.assert_close(dgu, C.swiglu_bwd(da, gu), atol=0, rtol=0)
    full = dgu.as_strided((T, 2 * F + pad), (2 * F + pad, 1))
    tail = full[:, 2 * F:].float()
    ref_tail = dgu.float() @ bt[:32].float().t()
    torch.testing.assert_close(tail[:, :32], ref_tail, atol=2e-2 * ref_tail.abs().max().item() + 1e-3, rtol=2e-2)
    assert torch.count_nonzero(tail[:, 32:]) == 0
    dgf = dgu.float()
    refB = mgB0.clone()
    refB[:F, :16] += dgf[:, :F].t() @ xa[:, :16].float()
    refB[F:, 16:] += dgf[:, F:].t() @ xa[:, 16:].float()
    tolB = 2e-2 * refB.abs().max().item()
    torch.testing.assert_close(mgB.float(), refB, atol=tolB, rtol=2e-2)
    assert torch.count_nonzero(mgB[:F, 16:]) == 0 and torch.count_nonzero(mgB[F:, :16]) == 0
    h = C.swiglu_fwd(gu).float()
    refA = mgA0 + 0.5 * (dyb.float().t() @ h)
    torch.testing.assert_close(mgA.float(), refA, atol=2e-2 * refA.abs().max().item(), rtol=2e-2)


@pytest.mark.parametrize("T,K,R,Rp", [(16384, 4096, 48, 64), (1000, 6144, 16, 64), (33, 128, 64, 64), (64, 256, 8, 16)])
def test_tail_gemm(C, T, K, R, Rp):
    """tail_gemm_ (csrc/kernels/swiglu_lora.hip): x[:, K:K+Rp] = x[:, :K] . Bm^T in place, zero past R."""
    torch.manual_seed(0)
    buf = bf(torch.randn(T, K + Rp + 8, device=DEV))
    x = buf[:, :K]
    bm = torch.zeros(Rp, K + 24, device=DEV, dtype=torch.bfloat16)
    bm[:R, :K] = bf(torch.randn(R, K, device=DEV) * 0.05)
    keep = buf[:, K + Rp:].clone()
    C.tail_gemm_(x, bm[:, :K], -(-R // 16), Rp)
    ref = x.float() @ bm[:R, :K].float().t()
    torch.testing.assert_close(buf[:, K:K + R].float(), ref, atol=2e-2 * ref.abs().max().item() + 1e-3, rtol=2e-2)
    assert torch.count_nonzero(buf[:, K + R:K + Rp]) == 0
    assert torch.equal(buf[:, K + Rp:], keep)  # nothing written past the tail


@pytest.mark.parametrize("V", [128256, 32000, 50257])
def test_cross_entropy_inplace(C, V):
    torch.manual_seed(0)
    n = 37
    logits = bf(torch.randn(n, V, device=DEV) * 3)
    labels = torch.randint(0, V, (n,), device=DEV)
    labels[3] = -100
    ref_logits = logits.float().clone().requires_grad_(True)
    nval = int((labels != -100).sum())
    loss_ref = torch.nn.functional.cross_entropy(ref_logits, labels, ignore_index=-100, reduction="sum") / nval
    loss_ref.backward()
    buf = logits.clone()
    loss_rows = C.ce_fwd_bwd_(buf, labels, 1.0 / nval, -100)
    torch.testing.assert_close(loss_rows.sum() / nval, loss_ref.detach(), atol=1e-3, rtol=1e-3)
    assert loss_rows[3].item() == 0.0
    torch.testing.assert_close(buf.float(), ref_logits.grad, atol=2e-3, rtol=5e-2)


@pytest.mark.parametrize("gdtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n", [3, 10_003, 1_000_001])
def test_adamw_flat(C, gdtype, n):
    """One-shot grid: tail-only (n < 4), one partial workgroup, many workgroups; tails n % 4 = 3 / 1."""
    torch.manual_seed(0)
    master = torch.randn(n, device=DEV)
    param = bf(master)
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    ref = master.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-2, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for step in range(1, 4):
        g = torch.randn(n, device=DEV).to(gdtype)
        ref.grad = g.float() * 0.5
        opt.step()
        stats = C.grad_sumsq(g, 0.0, 0.5)  # no clip, scale 0.5
        C.adamw_(param, master, m, v, g, 1e-2, 0.9, 0.95, 1e-8, 0.1, step, stats[1:2])
        torch.testing.assert_close(stats[0], (g.float() ** 2).sum(), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(master, ref.detach(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(param.float(), bf(ref.detach()).float(), atol=1e-2, rtol=1e-2)


@pytest.mark.parametrize("gdtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("n,offset", [(7, 0), (4_000_037, 0), (4_000_037, 1), (40_000_000, 0)])
def test_grad_sumsq_paths(C, gdtype, n, offset):
    """16-byte vector path (aligned), element path (offset view), tails, multi-iteration grids vs fp64."""
    torch.manual_seed(1)
    base = torch.randn(n + offset, device=DEV).to(gdtype)
    g = base[offset:]
    stats = C.grad_sumsq(g, 0.0, 1.0)
    ref = (g.double() ** 2).sum()
    assert abs(stats[0].item() - ref.item()) <= 1e-5 * ref.item() + 1e-3


@pytest.mark.parametrize("cdtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("splits", ["2", "4", "auto"])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_wgrad_split(C, cdtype, splits, beta):
    """Split-K weight gradient (ops.linear.wgrad_mm: batched GEMM into fp32 partials + splitk_sum_) on the
    operands of the production paths (dy^T as a transposed view, x transposed or as stored) vs fp32.
    256 x 768 = 3 tiles of a wide-input shape: "auto" splits it 2 ways at _WAVE = 2 (patched), as down dW
    is split at 256."""
    from finetune_controller_amd.ops import linear as L
    torch.manual_seed(5)
    T, M, N = 1024, 256, 768
    dy = (torch.rand(T, M, device=DEV) * 2 - 1).to(torch.bfloat16)
    x = (torch.rand(T, N, device=DEV) * 2 - 1).to(torch.bfloat16)
    old, old_split = L._WAVE, L._DW_SPLIT
    L._WAVE = 2
    try:
        assert L.dw_splits(M, N, T, splits) == (2 if splits == "auto" else int(splits))
        L._DW_SPLIT = splits
        tol = 2e-2 * (T ** 0.5) / 8 if cdtype == torch.bfloat16 else 1e-3 * (T ** 0.5) / 8
        for b in (x, L.transpose2d(x).t()):
            c = torch.randn(M, N, device=DEV).to(cdtype)
            ref = beta * c.float() + dy.float().t() @ x.float()
            L.wgrad_mm(c, dy.t(), b, beta)
            torch.testing.assert_close(c.float(), ref, atol=tol, rtol=1e-2 if cdtype == torch.bfloat16 else 1e-4)
    finally:
        L._WAVE = old
        L._DW_SPLIT = old_split  # (later tests keep the default "auto" split-K coverage)


def test_grad_clip_coef(C):
    g = torch.full((4096,), 0.5, device=DEV)
    stats = C.grad_sumsq(g, 1.0, 1.0)
    norm = math.sqrt(4096 * 0.25)
    assert abs(stats[1].item() - 1.0 / norm) < 1e-4


def test_nf4_roundtrip(C):
    from finetune_controller_amd.ops import nf4

    torch.manual_seed(0)
    w = bf(torch.randn(256, 512, device=DEV) * 0.02)
    q = nf4.NF4Weight.quantize(w)
    deq = q.dequantize()
    ref = nf4.dequantize_reference(q)
    torch.testing.assert_close(deq.float(), ref.float(), atol=1e-3, rtol=1e-2)
    # NF4 error bound: half the widest code gap times absmax
    assert (deq.float() - w.float()).abs().max().item() < 0.2 * w.abs().max().item()


def test_lora_merge(C):
    torch.manual_seed(0)
    W = bf(torch.randn(384, 256, device=DEV))
    A = bf(torch.randn(16, 256, device=DEV) * 0.1)
    B = bf(torch.randn(384, 16, device=DEV) * 0.1)
    ref = W.float() + 2.0 * (B.float() @ A.float())
    C.lora_merge_(W, A, B, 2.0, 0)
    torch.testing.assert_close(W.float(), ref, atol=3e-2, rtol=1e-2)


@pytest.mark.parametrize("B,S,H,KV,D,causal,window", [
    (2, 256, 8, 2, 128, True, 0),
    (1, 768, 4, 4, 128, False, 0),
    (1, 1024, 8, 2, 128, True, 0),
    (1, 512, 8, 2, 128, True, 192),
    (2, 256, 4, 4, 64, True, 0),
    (1, 1024, 8, 2, 64, True, 0),
    (1, 512, 8, 2, 64, False, 0),
    (1, 768, 8, 4, 64, True, 320),
])
def test_flash_attention_fwd_bwd(C, B, S, H, KV, D, causal, window):
    from finetune_controller_amd.ops.attention import _FlashPacked, attention_reference

    torch.manual_seed(0)
    W = (H + 2 * KV) * D
    qkv = bf(torch.randn(B * S, W, device=DEV))
    scale = 1.0 / math.sqrt(D)
    ref_in = qkv.float().clone().requires_grad_(True)
    ref = attention_reference(ref_in, B, S, H, KV, D, causal, window, scale)
    x = qkv.clone().requires_grad_(True)
    out = _FlashPacked.apply(x, B, S, H, KV, D, causal, window, scale, 0, 0)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    dout = bf(torch.randn(B * S, H * D, device=DEV))
    ref.backward(dout.float())
    out.backward(dout)
    g, gr = x.grad.float(), ref_in.grad
    # per-part relative error (dq | dk | dv)
    for lo, hi in ((0, H * D), (H * D, (H + KV) * D), ((H + KV) * D, W)):
        err = (g[:, lo:hi] - gr[:, lo:hi]).abs().max().item()
        mag = gr[:, lo:hi].abs().max().item()
        assert err <= 2e-2 * mag + 2e-2, (lo, err, mag)


@pytest.mark.parametrize("positions", [False, True])
def test_flash_bwd_rope_epilogue(C, positions):
    """flash_bwd with rope_cos / rope_sin: dq and dk leave inverse-rotated (the gradient w.r.t. the
    un-rotated q / k, csrc/kernels/flash_attn_bwd.hip rope_inv_rows), dv untouched -- against the plain
    kernel's dq / dk rotated back in fp32 torch (HF rotate_half, position = row in sequence or an
    explicit int32 [B*S] table)."""
    from finetune_controller_amd.ops.attention import _split

    torch.manual_seed(0)
    B, S, H, KV, D = 2, 512, 8, 2, 128
    W = (H + 2 * KV) * D
    qkv = bf(torch.randn(B * S, W, device=DEV))
    scale = 1.0 / math.sqrt(D)
    q, k, v = _split(qkv, B, S, H, KV, D)
    o, lse = C.flash_fwd(q, k, v, B, S, H, KV, D, scale, True, 0, 0, None)
    do = bf(torch.randn(B * S, H * D, device=DEV))
    inv = 1.0 / (10000.0 ** (torch.arange(0, 64, device=DEV, dtype=torch.float32) / 64))
    ang = torch.arange(4096, device=DEV, dtype=torch.float32)[:, None] * inv[None]
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    pos = (torch.randint(0, 4096, (B * S,), device=DEV, dtype=torch.int32) if positions else None)
    outs = []
    for rope in (False, True):
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = _split(dqkv, B, S, H, KV, D)
        C.flash_bwd(q, k, v, o, do, lse, dq, dk, dv, B, S, H, KV, D, scale, True, 0, None, None, -1,
                    cos if rope else None, sin if rope else None, pos if rope else None)
        outs.append(dqkv.float())
    plain, fused = outs
    p_ = pos.long() if positions else torch.arange(S, device=DEV).repeat(B)
    c, sn = cos[p_], sin[p_]                                        # [B*S, 64]
    ref = plain.clone()
    for h in range(H + KV):                                         # q and k heads
        g1, g2 = plain[:, h * D:h * D + 64], plain[:, h * D + 64:(h + 1) * D]
        ref[:, h * D:h * D + 64] = g1 * c + g2 * sn
        ref[:, h * D + 64:(h + 1) * D] = g2 * c - g1 * sn
    err = (fused - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err              # one bf16 rounding of a rotated value
    torch.testing.assert_close(fused[:, (H + KV) * D:], plain[:, (H + KV) * D:], atol=0, rtol=0)  # dv


@pytest.mark.parametrize("method", ["lora", "full"])
def test_llama_rope_grad_handoff(C, monkeypatch, method):
    """RoPE's producer on the HIP path (head_dim 128: the LoRA qkv projection, or the standalone op of
    full fine-tuning) hands its backward to the flash backward (ops.attention.RopeGrad): the handoff is
    taken, and every gradient of a step matches the same step with the separate inverse-rotation pass
    (ROPE_BWD_FUSE off) to bf16 rounding."""
    import finetune_controller_amd.ops.attention as att
    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import ModelConfig

    cfg = ModelConfig("llama", 512, 512, 2, 4, 2, 1024, 1024, 10000.0, name="llama-rope-test")  # head_dim 128
    torch.manual_seed(0)
    m = build_model(cfg, LoRAConfig(r=16, alpha=32) if method == "lora" else None, device=DEV, dtype=torch.bfloat16)
    m.init_weights(seed=5)
    if method == "lora":
        m.freeze_base()
        g = torch.Generator(device=DEV).manual_seed(1)
        with torch.no_grad():
            for layer in m.layers:
                for p in layer.lora.values():
                    for _, _, B_s in p.segment_tensors():
                        B_s.data.normal_(0, 0.05, generator=g)
    ids = torch.randint(0, cfg.vocab_size, (2, 512), device=DEV)
    labels = torch.roll(ids, -1, 1)
    made = []
    orig = att.RopeGrad.__init__

    def spy(self, *a):
        orig(self, *a)
        made.append(self)

    monkeypatch.setattr(att.RopeGrad, "__init__", spy)
    monkeypatch.setenv("FTC_KERNELS", "hip")
    grads = {}
    for fuse in (True, False):
        monkeypatch.setattr(att, "ROPE_BWD_FUSE", fuse)
        made.clear()
        for p in m.parameters():
            p.grad = None
        m(ids, labels).backward()
        assert made and all(h.taken == fuse for h in made), [h.taken for h in made]
        grads[fuse] = {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None}
    assert grads[True].keys() == grads[False].keys() and grads[True]
    for n, ref in grads[False].items():
        den = ref.norm().item()
        err = (grads[True][n] - ref).norm().item() / max(den, 1e-30)
        assert err < 2e-2, (n, err)


@pytest.mark.parametrize("B,S,H,KV,D,window,docs", [
    (1, 1000, 8, 2, 128, 0, False),
    (1, 3000, 8, 2, 128, 0, False),
    (2, 1000, 8, 4, 64, 0, False),
    (1, 3000, 8, 2, 64, 512, False),
    (1, 1000, 8, 2, 128, 300, False),
    (2, 700, 4, 2, 128, 0, True),
])
@pytest.mark.parametrize("causal", [True, False])
def test_flash_tail_lengths(C, B, S, H, KV, D, window, docs, causal):
    """S not a multiple of the 256-row tile: attention_packed takes the tail-padded flash path (not
    SDPA) and matches the fp32 reference, forward and backward -- causal (pads never visible) and
    non-causal (pad keys masked in the kernels through kv_valid)."""
    from finetune_controller_amd.ops import attention as A

    if docs and not causal:
        pytest.skip("document masking is causal")
    assert not A.flash_supported(D, S) and A.flash_usable(D, S, causal)
    torch.manual_seed(0)
    W = (H + 2 * KV) * D
    qkv = bf(torch.randn(B * S, W, device=DEV))
    seg = None
    if docs:
        ids = torch.randint(3, 100, (B, S), device=DEV)
        ids[0, 211] = ids[0, 650] = ids[1, 300] = 2
        seg = A.segments_from_eos(ids, 2)
    scale = 1.0 / math.sqrt(D)
    ref_in = qkv.float().clone().requires_grad_(True)
    ref = A.attention_reference(ref_in, B, S, H, KV, D, causal, window, scale, docs=seg)
    x = qkv.clone().requires_grad_(True)
    out = A.attention_packed(x, B, S, H, KV, D, causal, window, scale, out_pad=64, grad_pad=64, docs=seg)
    assert out.grad_fn is not None and "PaddedTail" in type(out.grad_fn).__name__
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    dout = bf(torch.randn(B * S, H * D, device=DEV))
    ref.backward(dout.float())
    out.backward(dout)
    g, gr = x.grad.float(), ref_in.grad
    for lo, hi in ((0, H * D), (H * D, (H + KV) * D), ((H + KV) * D, W)):
        err = (g[:, lo:hi] - gr[:, lo:hi]).abs().max().item()
        mag = gr[:, lo:hi].abs().max().item()
        assert err <= 2e-2 * mag + 2e-2, (lo, err, mag)


@pytest.mark.parametrize("B,S,H,KV,D,window,causal", [
    (2, 512, 8, 2, 96, 0, True),
    (1, 700, 4, 4, 80, 0, True),
    (1, 512, 6, 2, 112, 200, True),
    (2, 300, 4, 2, 96, 0, False),
    (1, 256, 4, 2, 32, 0, True),
])
def test_flash_head_dim_padded(C, B, S, H, KV, D, window, causal):
    """head_dim outside the kernels' {64, 128} (80 / 96 / 112 / 32): attention_packed zero-pads every head
    to the next kernel head_dim and runs the flash kernels (not SDPA), forward and backward equal to the
    fp32 reference at the real D's softmax scale."""
    from finetune_controller_amd.ops import attention as A

    assert not A.flash_supported(D, S) and A.flash_usable(D, S, causal)
    torch.manual_seed(0)
    W = (H + 2 * KV) * D
    qkv = bf(torch.randn(B * S, W + 64, device=DEV))[:, :W]  # a column view, as the qkv GEMM hands it
    scale = 1.0 / math.sqrt(D)
    ref_in = qkv.float().clone().requires_grad_(True)
    ref = A.attention_reference(ref_in, B, S, H, KV, D, causal, window, scale)
    x = qkv.detach().clone().requires_grad_(True)
    out = A.attention_packed(x, B, S, H, KV, D, causal, window, out_pad=64, grad_pad=64)
    assert out.grad_fn is not None and "PaddedTail" in type(out.grad_fn).__name__
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    dout = bf(torch.randn(B * S, H * D, device=DEV))
    ref.backward(dout.float())
    out.backward(dout)
    g, gr = x.grad.float(), ref_in.grad
    for lo, hi in ((0, H * D), (H * D, (H + KV) * D), ((H + KV) * D, W)):
        rel = ((g[:, lo:hi] - gr[:, lo:hi]).norm() / gr[:, lo:hi].norm()).item()
        assert rel < 1.5e-2, (lo, rel)


def test_flash_lse(C):
    torch.manual_seed(1)
    B, S, H, KV, D = 1, 256, 4, 2, 128
    qkv = bf(torch.randn(B * S, (H + 2 * KV) * D, device=DEV))
    q, k, v = qkv[:, :H * D], qkv[:, H * D:(H + KV) * D], qkv[:, (H + KV) * D:]
    o, lse = C.flash_fwd(q, k, v, B, S, H, KV, D, 1 / math.sqrt(D), True, 0)
    qf = q.float().view(S, H, D).transpose(0, 1)
    kf = k.float().view(S, KV, D).transpose(0, 1).repeat_interleave(H // KV, 0)
    s = qf @ kf.transpose(-1, -2) / math.sqrt(D)
    s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=DEV), 1), float("-inf"))
    torch.testing.assert_close(lse.view(H, S), torch.logsumexp(s, -1), atol=2e-3, rtol=1e-3)


@pytest.mark.parametrize("window,aug,ckpt", [(0, "1", False), (0, "0", False), (96, "1", False), (0, "1", True)])
def test_llama_lora_step_hip_matches_torch_path(C, monkeypatch, window, aug, ckpt):
    """Whole decoder with LoRA on the HIP path (flash attention, fused norms, SwiGLU with fused LoRA
    tails, augmented LoRA GEMMs over padded producer buffers; optionally per-layer activation
    checkpointing, i.e. the forward recomputed inside backward) against the stock-PyTorch path."""
    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import ModelConfig

    cfg = ModelConfig("llama", 512, 256, 2, 4, 2, 512, 512, 10000.0, sliding_window=window, name="llama-test")
    lc = LoRAConfig(r=8, alpha=16)
    torch.manual_seed(0)
    models = []
    for i in range(2):
        m = build_model(cfg, lc, device=DEV, dtype=torch.bfloat16, checkpoint_layers=ckpt and i == 0)
        m.init_weights(seed=5)
        m.freeze_base()
        models.append(m)
    g = torch.Generator(device=DEV).manual_seed(1)
    for layer in models[0].layers:
        assert set(layer.aug) == {"qkv", "o", "gu", "down"}
        for p in layer.lora.values():
            for _, _, B_s in p.segment_tensors():
                B_s.data.normal_(0, 0.05, generator=g)
    with torch.no_grad():
        for p0, p1 in zip(models[0].parameters(), models[1].parameters()):
            p1.copy_(p0)
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device=DEV)
    labels = torch.roll(ids, -1, 1)
    monkeypatch.setenv("FTC_LORA_AUG", aug)
    losses, grads = [], []
    for mode, m in (("hip", models[0]), ("torch", models[1])):
        monkeypatch.setenv("FTC_KERNELS", mode)
        loss = m(ids, labels)
        loss.backward()
        losses.append(loss.float().item())
        grads.append({n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None})
    assert abs(losses[0] - losses[1]) < 2e-2 * abs(losses[1]), losses
    assert grads[0].keys() == grads[1].keys() and len(grads[0]) > 0
    bad = []
    for n in grads[0]:
        a, b = grads[0][n], grads[1][n]
        err = (a - b).abs().max().item()
        if err > 5e-2 * b.abs().max().item() + 1e-3:
            bad.append((n, round(err, 5), round(b.abs().max().item(), 5)))
    assert not bad, bad


@pytest.mark.parametrize("method", ["lora", "full"])
def test_llama_hip_vs_fp32_model_reference(C, monkeypatch, method):
    """Whole-model parity against an fp32 reference (the same weights upcast, stock-torch ops in fp32):
    per-tensor relative L2 error ||g - g32|| / ||g32|| of EVERY gradient (each LoRA segment separately,
    so a scale error confined to one small tensor cannot hide behind a global max).  Calibration: the
    stock-PyTorch bf16 path's own error against the same reference -- the HIP path must be within 2x of
    it (+ 1e-3) on every tensor, and within 5e-2 absolute."""
    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import ModelConfig

    cfg = ModelConfig("llama", 512, 256, 2, 4, 2, 512, 512, 10000.0, name="llama-test")
    lc = LoRAConfig(r=8, alpha=16) if method == "lora" else None
    torch.manual_seed(0)
    models = {}
    for key, dt in (("hip", torch.bfloat16), ("torch", torch.bfloat16), ("fp32", torch.float32)):
        m = build_model(cfg, lc, device=DEV, dtype=dt)
        m.init_weights(seed=5)
        if lc is not None:
            m.freeze_base()
        models[key] = m
    g = torch.Generator(device=DEV).manual_seed(1)
    with torch.no_grad():
        if lc is not None:
            for layer in models["hip"].layers:
                for p in layer.lora.values():
                    for _, _, B_s in p.segment_tensors():
                        B_s.data.normal_(0, 0.05, generator=g)
        for k in ("torch", "fp32"):
            for p0, p1 in zip(models["hip"].parameters(), models[k].parameters()):
                p1.copy_(p0)  # fp32: the bf16 weights upcast exactly
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device=DEV)
    labels = torch.roll(ids, -1, 1)
    losses, grads = {}, {}
    for key, mode in (("hip", "hip"), ("torch", "torch"), ("fp32", "torch")):
        monkeypatch.setenv("FTC_KERNELS", mode)
        m = models[key]
        loss = m(ids, labels)
        loss.backward()
        losses[key] = loss.double().item()
        grads[key] = {n: p.grad.double().clone() for n, p in m.named_parameters() if p.grad is not None}
    assert grads["hip"].keys() == grads["fp32"].keys() == grads["torch"].keys() and grads["hip"]
    assert abs(losses["hip"] - losses["fp32"]) <= max(2 * abs(losses["torch"] - losses["fp32"]), 1e-3 * losses["fp32"])
    bad = []
    for n, ref in grads["fp32"].items():
        den = ref.norm().item()
        if den == 0:
            continue
        e_hip = (grads["hip"][n] - ref).norm().item() / den
        e_bf16 = (grads["torch"][n] - ref).norm().item() / den
        if e_hip > 2 * e_bf16 + 1e-3 or e_hip > 5e-2:
            bad.append((n, round(e_hip, 5), round(e_bf16, 5)))
    assert not bad, bad


def test_llama3_8b_layer_shape_parity(C, monkeypatch):
    """Production-shape numerics (VERDICT r4 Next #6): two Llama-3-8B decoder layers (d 4096, H32 / KV8 x 128,
    F 14336, RoPE 5e5) at S = 4096, B = 1, LoRA r16 / alpha 32 on all seven projections -- the headline's
    augmented GEMM strides ([x | s x A^T] with 64 pad columns), fused norms / RoPE / SwiGLU tails, flash
    fwd / bwd at the headline tile -- through the HIP path against the same weights in fp32 stock torch.
    Per-tensor relative L2 of the final hidden state, of dx (the embedding gradient: the first layer's
    input gradient scattered by token id; the embedding is made trainable for this) and of every LoRA
    gradient (each of the seven projections' A and B separately).  Bounds: within 2x the stock-PyTorch bf16
    path's own error + 1e-3, and 5e-2 absolute (measured: the second layer's q / k adapters carry the largest
    error on BOTH bf16 paths, 3.2e-2 HIP vs 3.7e-2 stock -- bf16 softmax-gradient noise at S = 4096).  A small vocabulary keeps the lm_head out of the way."""
    import time

    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import ModelConfig

    t0 = time.time()
    cfg = ModelConfig("llama", 2048, 4096, 2, 32, 8, 14336, 4096, 500000.0, name="llama3-8b-2layer")
    lc = LoRAConfig(r=16, alpha=32)
    torch.manual_seed(0)
    models = {}
    for key, dt in (("hip", torch.bfloat16), ("torch", torch.bfloat16), ("fp32", torch.float32)):
        m = build_model(cfg, lc, device=DEV, dtype=dt)
        m.init_weights(seed=7)
        m.freeze_base()
        m.embed.requires_grad_(True)
        models[key] = m
    g = torch.Generator(device=DEV).manual_seed(2)
    with torch.no_grad():
        for layer in models["hip"].layers:  # non-zero B so every adapter path carries signal
            for p in layer.lora.values():
                for _, _, B_s in p.segment_tensors():
                    B_s.data.normal_(0, 0.02, generator=g)
        for k in ("torch", "fp32"):
            for p0, p1 in zip(models["hip"].parameters(), models[k].parameters()):
                p1.copy_(p0)
            models[k].invalidate_transposed()
    ids = torch.randint(0, cfg.vocab_size, (1, 4096), device=DEV)
    labels = torch.roll(ids, -1, 1)
    hidden, grads, losses = {}, {}, {}
    for key, mode in (("hip", "hip"), ("torch", "torch"), ("fp32", "torch")):
        monkeypatch.setenv("FTC_KERNELS", mode)
        m = models[key]
        with torch.no_grad():
            hidden[key] = m.hidden(ids).double()
        loss = m(ids, labels)
        loss.backward()
        losses[key] = loss.double().item()
        grads[key] = {n: p.grad.double() for n, p in m.named_parameters() if p.grad is not None}
        torch.cuda.synchronize()
    assert grads["hip"].keys() == grads["fp32"].keys() and "embed" in grads["hip"]
    assert sum(".lora." in n for n in grads["hip"]) == 2 * 4 * 2  # A and B of 4 packed projections x 2 layers

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()

    def segments(key):  # every LoRA gradient per projection segment (q / k / v, gate / up, ...), + the rest
        out = {n: t for n, t in grads[key].items() if ".lora." not in n}
        for li, layer in enumerate(models[key].layers):
            for pname, pair in layer.lora.items():
                i = row = 0
                for seg, nrows in pair.segments:
                    if seg in pair.names:
                        out[f"{li}.{seg}.A"] = pair.A.grad[i * pair.r:(i + 1) * pair.r].double()
                        out[f"{li}.{seg}.B"] = pair.B.grad[row:row + nrows, i * pair.r:(i + 1) * pair.r].double()
                        i += 1
                    row += nrows
        return out

    seg = {k: segments(k) for k in grads}
    assert sum(n.endswith((".A", ".B")) for n in seg["hip"]) == 2 * 7 * 2  # 7 projections x A, B x 2 layers
    rows = {"hidden": (rel(hidden["hip"], hidden["fp32"]), rel(hidden["torch"], hidden["fp32"]))}
    for n, ref in seg["fp32"].items():
        if ref.norm().item() == 0:
            continue
        rows[n] = (rel(seg["hip"][n], ref), rel(seg["torch"][n], ref))
    bad = [(n, round(e, 5), round(e16, 5)) for n, (e, e16) in rows.items() if e > 2 * e16 + 1e-3 or e > 5e-2]
    assert not bad, bad
    assert abs(losses["hip"] - losses["fp32"]) <= max(2 * abs(losses["torch"] - losses["fp32"]), 1e-3 * losses["fp32"])
    assert time.time() - t0 < 60


def test_native_rccl_engine_world1(C):
    """csrc/comm engine on one rank: communicator bootstrap through c10d, every collective, event
    ordering against the current stream.  The 2-rank gradient equivalence of the bucketer over real
    RCCL (both engines) is tests/test_distributed.py::test_ddp_rccl_matches_per_rank_sum."""
    import os

    import torch.distributed as dist

    from finetune_controller_amd.parallel.comm import NativeComm

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device(DEV, 0))
    try:
        comm = NativeComm()
        for dt in (torch.float32, torch.bfloat16):
            t = torch.randn(4099, device=DEV).to(dt)
            ref = t.clone()
            t.mul_(1.0)  # queued on the current stream before the collective
            comm.all_reduce_async(t).wait()
            t.add_(1)  # ordered after it on the device
            torch.cuda.synchronize()
            torch.testing.assert_close(t, ref + 1)
        b = torch.arange(64, device=DEV, dtype=torch.float32)
        comm.broadcast_async(b, 0).wait()
        out = torch.empty(64, device=DEV)
        comm.all_gather_async(out, b).wait()
        rs = torch.empty(64, device=DEV)
        comm.reduce_scatter_async(rs, b).wait()
        torch.cuda.synchronize()
        assert torch.equal(out, b) and torch.equal(rs, b)
        assert comm.bench_all_reduce(torch.empty(1 << 20, device=DEV), 3) > 0
        comm.reset()
        comm.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("M", [1, 17, 64, 100])
def test_nf4_fused_gemm_matches_dequant(C, M):
    from finetune_controller_amd.ops import nf4

    torch.manual_seed(M)
    N, K = 96, 512
    W = bf(torch.randn(N, K, device=DEV) * 0.05)
    qw = nf4.NF4Weight.quantize(W)
    x = bf(torch.randn(M, K, device=DEV))
    ref = x.float() @ qw.dequantize().float().t()
    y = C.nf4_linear(x, qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, N, qw.block, qw.block2)
    torch.testing.assert_close(y.float(), ref, atol=2e-2, rtol=2e-2)
    # the ops-level dispatcher takes the fused path at this M
    torch.testing.assert_close(nf4.nf4_matmul(x, qw).float(), ref, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("N,K", [(192, 320), (512, 1408), (256, 4160)])
def test_nf4_dequantize_into_rows_and_transposed(C, N, K):
    """Row and transposed (64 x 128 LDS tile; K % 128 == 64 ends in a half tile) decodes, bitwise the
    reference dequantisation, nothing written outside the views."""
    from finetune_controller_amd.ops import nf4

    torch.manual_seed(3)
    qw = nf4.NF4Weight.quantize(bf(torch.randn(N, K, device=DEV) * 0.05))
    ref = qw.dequantize()
    buf = torch.full((N, K + 64), 7.0, device=DEV, dtype=torch.bfloat16)
    C.nf4_dequantize_into(qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, buf[:, :K], N, K, 64,
                          qw.block2, False)
    assert torch.equal(buf[:, :K], ref) and (buf[:, K:] == 7.0).all()
    bufT = torch.full((K, N + 64), 7.0, device=DEV, dtype=torch.bfloat16)
    C.nf4_dequantize_into(qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, bufT[:, :N], N, K, 64,
                          qw.block2, True)
    assert torch.equal(bufT[:, :N], ref.t()) and (bufT[:, N:] == 7.0).all()


@pytest.mark.parametrize("with_b", [True, False])
def test_nf4_dequantize_aug_fills_rank_parts(C, with_b):
    """One launch writes W (or W^T) plus the rank-r operand parts the QLoRA augmented GEMMs need: B into
    its columns and s*A into its rows (transposed: (s A)^T into columns) -- bitwise what the separate
    copy / torch.mul kernels wrote, and nothing outside the views."""
    from finetune_controller_amd.ops import nf4

    torch.manual_seed(4)
    N, K, R, Rp, s = 192, 320, 48, 64, 2.0
    qw = nf4.NF4Weight.quantize(bf(torch.randn(N, K, device=DEV) * 0.05))
    ref = qw.dequantize()
    A, B = bf(torch.randn(R, K, device=DEV)), bf(torch.randn(N, R, device=DEV))
    fwd = torch.full((N + Rp, K + Rp), 7.0, device=DEV, dtype=torch.bfloat16)
    C.nf4_dequantize_aug(qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, fwd[:N, :K], N, K, 64, qw.block2,
                         False, B if with_b else None, fwd[:N, K:K + R] if with_b else None, A, fwd[N:N + R, :K], s)
    want = torch.full_like(fwd, 7.0)
    want[:N, :K] = ref
    if with_b:
        want[:N, K:K + R] = B
    want[N:N + R, :K] = A * s
    assert torch.equal(fwd, want)
    bwdT = torch.full((K, N + Rp), 7.0, device=DEV, dtype=torch.bfloat16)
    Bp = torch.full((N, Rp), 7.0, device=DEV, dtype=torch.bfloat16)
    C.nf4_dequantize_aug(qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, bwdT[:, :N], N, K, 64, qw.block2,
                         True, B if with_b else None, Bp[:, :R] if with_b else None, A, bwdT[:, N:N + R], s)
    wantT = torch.full_like(bwdT, 7.0)
    wantT[:, :N] = ref.t()
    wantT[:, N:N + R] = (A * s).t()
    assert torch.equal(bwdT, wantT)
    assert torch.equal(Bp[:, :R], B) if with_b else bool((Bp == 7.0).all())
    assert (Bp[:, R:] == 7.0).all()


def test_qlora_step_hip_matches_torch_path(C, monkeypatch):
    """Mistral-style trunk (sliding window) in QLoRA: NF4 base dequantised into the augmented operands
    (forward) and their transposed form (backward) vs the stock-PyTorch path on the same NF4 weights."""
    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import ModelConfig
    from finetune_controller_amd.ops.nf4 import quantize_model_

    cfg = ModelConfig("llama", 512, 256, 2, 4, 2, 512, 1024, 10000.0, sliding_window=128, name="mistral-test")
    torch.manual_seed(0)
    models = []
    for _ in range(2):
        m = build_model(cfg, LoRAConfig(r=8, alpha=16), device=DEV, dtype=torch.bfloat16)
        m.init_weights(seed=9)
        m.freeze_base()
        models.append(m)
    g = torch.Generator(device=DEV).manual_seed(2)
    for layer in models[0].layers:
        for p in layer.lora.values():
            for _, _, B_s in p.segment_tensors():
                B_s.data.normal_(0, 0.05, generator=g)
    with torch.no_grad():
        for p0, p1 in zip(models[0].parameters(), models[1].parameters()):
            p1.copy_(p0)
    for m in models:
        quantize_model_(m)
    ids = torch.randint(0, cfg.vocab_size, (2, 512), device=DEV)
    labels = torch.roll(ids, -1, 1)
    out = []
    for mode, m in (("hip", models[0]), ("torch", models[1])):
        monkeypatch.setenv("FTC_KERNELS", mode)
        loss = m(ids, labels)
        loss.backward()
        out.append((loss.float().item(), {n: p.grad.float().clone() for n, p in m.named_parameters()
                                          if p.grad is not None}))
    (l0, g0), (l1, g1) = out
    assert abs(l0 - l1) < 2e-2 * abs(l1), (l0, l1)
    bad = [n for n in g0 if (g0[n] - g1[n]).abs().max() > 5e-2 * g1[n].abs().max() + 1e-3]
    assert not bad and len(g0) > 0, bad


@pytest.mark.parametrize("T,M,R,transposed,col0", [(1024, 4096, 16, False, 0), (512, 1024, 48, False, 16),
                                                   (256, 14336, 16, True, 0), (4096, 128, 64, True, 8),
                                                   (64, 256, 32, False, 0)])
def test_lora_wgrad_matches_fp32(C, T, M, R, transposed, col0):
    """out [M, R] += alpha X^T Y through csrc/kernels/lora_wgrad.hip (split-T MFMA + split reduction), with
    X / Y as column views of wider row-padded buffers (the augmented-GEMM operands) and out either a
    row-major [M, R] block or the transposed view of an [R, M] gradient (dA)."""
    torch.manual_seed(0)
    Xbuf = bf(torch.randn(T, M + 64, device=DEV))
    Ybuf = bf(torch.randn(T, col0 + R + 24, device=DEV))
    X, Y = Xbuf[:, :M], Ybuf[:, col0:col0 + R]
    assert C.lora_wgrad_ok(X, Y, R)
    if transposed:
        base = bf(torch.randn(R, M, device=DEV))
        out = base.t()
    else:
        base = bf(torch.randn(M, R + 8, device=DEV))
        out = base[:, :R]
    before = out.float().clone()
    C.lora_wgrad_(out, X, Y, R, 0.5, 1.0)
    ref = before + 0.5 * (X.float().t() @ Y.float())
    torch.testing.assert_close(out.float(), ref, atol=0.05 + 2e-3 * math.sqrt(T), rtol=1e-2)


def test_lora_wgrad_block_diagonal_segments(C):
    """Packed q|k|v dB in one launch: rows of each segment use their own 16 columns of Y and of out; the
    off-diagonal blocks of out are not touched."""
    torch.manual_seed(0)
    T, R = 512, 16
    bounds = [(0, 512), (512, 640), (640, 768)]
    X = bf(torch.randn(T, 768 + 64, device=DEV))[:, :768]
    Y = bf(torch.randn(T, 64, device=DEV))  # s x A^T tail: 3 x 16 used columns + zero pad
    out = bf(torch.randn(768, 3 * R, device=DEV))
    before = out.float().clone()
    C.lora_wgrad_(out, X, Y, R, 1.0, 1.0, [b[1] for b in bounds], [0, 16, 32], [0, 16, 32])
    ref = before.clone()
    for i, (r0, r1) in enumerate(bounds):
        ref[r0:r1, 16 * i:16 * i + 16] += X[:, r0:r1].float().t() @ Y[:, 16 * i:16 * i + 16].float()
    torch.testing.assert_close(out.float(), ref, atol=0.1, rtol=1e-2)


@pytest.mark.parametrize("rows,cols,pad", [(16384, 4096, 0), (4096, 14336, 64), (200, 72, 8), (8, 8, 0),
                                           (136, 4160, 0)])
def test_transpose2d(C, rows, cols, pad):
    """csrc/kernels/transpose.hip: exact copy of x^T for row views (padded strides, partial edge tiles)."""
    torch.manual_seed(0)
    buf = bf(torch.randn(rows, cols + pad, device=DEV))
    x = buf[:, :cols]
    y = C.transpose2d(x)
    assert y.shape == (cols, rows) and y.is_contiguous()
    assert torch.equal(y, x.t())
    out = torch.empty(cols, rows, device=DEV, dtype=torch.bfloat16)
    assert C.transpose2d(x, out).data_ptr() == out.data_ptr() and torch.equal(out, x.t())


def test_full_ft_steps_hip_match_torch_path(C, monkeypatch):
    """Full fine-tuning on the HIP path -- TN input-gradient GEMMs through per-step W^T copies, weight
    gradients with the activation transposed (csrc/kernels/transpose.hip), flat AdamW -- against the
    stock-PyTorch path over two optimizer steps (the W^T cache must follow the in-place updates)."""
    from finetune_controller_amd.models import build_model
    from finetune_controller_amd.models.config import ModelConfig
    from finetune_controller_amd.train.optim import FlatAdamW

    cfg = ModelConfig("llama", 512, 256, 2, 4, 2, 512, 512, 10000.0, name="llama-test")
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device=DEV)
    labels = torch.roll(ids, -1, 1)
    results = {}
    for mode in ("hip", "torch"):
        monkeypatch.setenv("FTC_KERNELS", mode)
        torch.manual_seed(0)
        m = build_model(cfg, None, device=DEV, dtype=torch.bfloat16)
        m.init_weights(seed=5)
        opt = FlatAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, max_grad_norm=1.0)
        losses = []
        for _ in range(3):
            opt.zero_grad()
            loss = m(ids, labels)
            loss.backward()
            opt.step()
            losses.append(loss.float().item())
        results[mode] = (losses, opt.param_flat.float().clone())
    (lh, ph), (lt, pt) = results["hip"], results["torch"]
    for a, b in zip(lh, lt):
        assert abs(a - b) < 2e-2 * abs(b), (lh, lt)
    assert lh[2] < lh[0]  # it trains
    # parameters after three AdamW steps: every element moved by ~lr per step; compare the drift
    err = (ph - pt).abs().max().item()
    assert err < 1e-2, err


def test_llama_fused_lora_mlp_matches_torch_path(C, monkeypatch):
    """The fused LoRA MLP block (ops/mlp.py: SwiGLU backward forming dB_gu / dA_down, augmented GEMMs)
    on adapters homed in FlatAdamW's flat gradient buffer, against the stock-PyTorch path: loss and
    every adapter gradient of a whole decoder."""
    import finetune_controller_amd.models.llama as llama_mod
    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import ModelConfig
    from finetune_controller_amd.train.optim import FlatAdamW

    cfg = ModelConfig("llama", 512, 256, 2, 4, 2, 1024, 512, 10000.0, name="llama-test")
    lc = LoRAConfig(r=16, alpha=32)
    calls = []
    real = llama_mod.lora_mlp
    monkeypatch.setattr(llama_mod, "lora_mlp", lambda *a, **k: calls.append(1) or real(*a, **k))
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device=DEV)
    labels = torch.roll(ids, -1, 1)
    res = {}
    for mode in ("hip", "torch"):
        monkeypatch.setenv("FTC_KERNELS", mode)
        torch.manual_seed(0)
        m = build_model(cfg, lc, device=DEV, dtype=torch.bfloat16)
        m.init_weights(seed=5)
        m.freeze_base()
        g = torch.Generator(device=DEV).manual_seed(1)
        for layer in m.layers:
            for p in layer.lora.values():
                for _, _, B_s in p.segment_tensors():
                    B_s.data.normal_(0, 0.05, generator=g)
        opt = FlatAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3)
        opt.zero_grad()
        loss = m(ids, labels)
        loss.backward()
        res[mode] = (loss.float().item(), opt.grad_flat.float().clone(), [(o, n) for o, n in opt.offsets])
    assert len(calls) == cfg.n_layers  # the fused block ran in every layer on the HIP path
    (lh, gh, offs), (lt, gt, _) = res["hip"], res["torch"]
    assert abs(lh - lt) < 2e-2 * abs(lt)
    bad = []
    for o, n in offs:
        a, b = gh[o:o + n], gt[o:o + n]
        if (a - b).abs().max().item() > 5e-2 * b.abs().max().item() + 1e-3:
            bad.append((o, n, (a - b).abs().max().item(), b.abs().max().item()))
    assert not bad, bad


@pytest.mark.parametrize("name", ["llama3.2-1b", "llama3.2-3b", "llama3-70b", "mistral-7b-v0.3", "llama3.1-8b"])
def test_llama_family_presets_hip_match_torch(C, monkeypatch, name):
    """One full-width layer of each Llama-trunk preset (head_dim 64 flash path, GQA 3:1, tied
    embeddings, Llama-3.1 rope scaling, the 70B width) with LoRA r=16 on adapters homed in a flat
    gradient buffer: HIP path (fused MLP block included) against the stock-PyTorch path."""
    import dataclasses

    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import get_config
    from finetune_controller_amd.train.optim import FlatAdamW

    cfg = dataclasses.replace(get_config(name), n_layers=1, max_seq_len=512)
    lc = LoRAConfig(r=16, alpha=32)
    ids = torch.randint(0, cfg.vocab_size, (1, 512), device=DEV)
    labels = torch.roll(ids, -1, 1)
    res = {}
    for mode in ("hip", "torch"):
        monkeypatch.setenv("FTC_KERNELS", mode)
        torch.manual_seed(0)
        m = build_model(cfg, lc, device=DEV, dtype=torch.bfloat16)
        m.init_weights(seed=5)
        m.freeze_base()
        g = torch.Generator(device=DEV).manual_seed(1)
        for layer in m.layers:
            for p in layer.lora.values():
                for _, _, B_s in p.segment_tensors():
                    B_s.data.normal_(0, 0.05, generator=g)
        opt = FlatAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3)
        opt.zero_grad()
        loss = m(ids, labels)
        loss.backward()
        res[mode] = (loss.float().item(), opt.grad_flat.float().clone(), list(opt.offsets))
        del m, opt
        torch.cuda.empty_cache()
    (lh, gh, offs), (lt, gt, _) = res["hip"], res["torch"]
    assert abs(lh - lt) < 2e-2 * abs(lt), (lh, lt)
    for o, n in offs:
        a, b = gh[o:o + n], gt[o:o + n]
        assert (a - b).abs().max().item() <= 5e-2 * b.abs().max().item() + 1e-3, (name, o, n)


def test_qlora_fused_mlp_matches_torch_path(C, monkeypatch):
    """QLoRA through the fused MLP block (NF4Proj: dequantised augmented / TN operands, SwiGLU backward
    forming dB_gu / dA_down) against the stock-PyTorch QLoRA path, adapters in flat gradient buffers."""
    import finetune_controller_amd.models.llama as llama_mod
    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import ModelConfig
    from finetune_controller_amd.ops.nf4 import quantize_model_
    from finetune_controller_amd.train.optim import FlatAdamW

    cfg = ModelConfig("llama", 512, 256, 2, 4, 2, 1024, 512, 10000.0, name="llama-test")
    calls = []
    real = llama_mod.lora_mlp
    monkeypatch.setattr(llama_mod, "lora_mlp", lambda *a, **k: calls.append(1) or real(*a, **k))
    ids = torch.randint(0, cfg.vocab_size, (2, 256), device=DEV)
    labels = torch.roll(ids, -1, 1)
    res = {}
    for mode in ("hip", "torch"):
        monkeypatch.setenv("FTC_KERNELS", mode)
        torch.manual_seed(0)
        m = build_model(cfg, LoRAConfig(r=16, alpha=32), device=DEV, dtype=torch.bfloat16)
        m.init_weights(seed=5)
        m.freeze_base()
        quantize_model_(m)
        g = torch.Generator(device=DEV).manual_seed(1)
        for layer in m.layers:
            for p in layer.lora.values():
                for _, _, B_s in p.segment_tensors():
                    B_s.data.normal_(0, 0.05, generator=g)
        opt = FlatAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3)
        opt.zero_grad()
        loss = m(ids, labels)
        loss.backward()
        res[mode] = (loss.float().item(), opt.grad_flat.float().clone(), list(opt.offsets))
    assert len(calls) == cfg.n_layers
    (lh, gh, offs), (lt, gt, _) = res["hip"], res["torch"]
    assert abs(lh - lt) < 2e-2 * abs(lt)
    for o, n in offs:
        a, b = gh[o:o + n], gt[o:o + n]
        assert (a - b).abs().max().item() <= 5e-2 * b.abs().max().item() + 1e-3, (o, n)


@pytest.mark.parametrize("method", ["lora", "full"])
def test_trainer_evaluate_hip_no_grad(C, tmp_path, method):
    """Trainer.evaluate on the HIP path: a forward under no_grad through the fused LoRA MLP / fused CE
    leaves every gradient buffer untouched, returns the same loss twice, and matches a training-mode
    forward of the same batch (the eval forward computes the same function)."""
    from finetune_controller_amd.train.trainer import Trainer, TrainConfig

    tr = Trainer(TrainConfig(model="llama-smoke", method=method, batch_size=2, seq_len=256, synthetic=True,
                             max_steps=1, eval_batches=2, checkpoint_path=str(tmp_path), resume=False,
                             device="cuda", save_model=False, warmup_steps=0))
    tr.train_step(1e-4)
    torch.cuda.synchronize()
    g0 = tr.opt.grad_flat.detach().clone()
    a, b = tr.evaluate(), tr.evaluate()
    torch.cuda.synchronize()
    assert torch.equal(tr.opt.grad_flat, g0)
    assert a == b and math.isfinite(a)
    batches = list(tr.eval_batches())
    ref = 0.0
    for x, y in batches:
        with torch.no_grad():
            ref += float(tr.model(x, y))  # training mode, no grad: same function as eval
    assert abs(a - ref / len(batches)) < 1e-3 * abs(a)
    tr.close()


def test_mnist_example_on_gpu(tmp_path):
    """The reference's example job runs on the MI355X worker (MIOpen convolutions, one process)."""
    from finetune_controller_amd.train import mnist

    last = mnist.run(mnist.build_parser().parse_args(
        ["--epochs", "1", "--train-size", "4000", "--test-size", "1000", "--log-interval", "50",
         "--dataset_path", str(tmp_path / "none"), "--checkpoint_path", str(tmp_path / "out")]))
    assert last["accuracy"] > 90.0


def _doc_ids(B, S, lens_per_row, eos=2):
    ids = torch.full((B, S), 5, dtype=torch.long)
    for b, lens in enumerate(lens_per_row):
        pos = 0
        for n in lens:
            pos += n
            if pos <= S:
                ids[b, pos - 1] = eos
    return ids.to(DEV)


@pytest.mark.parametrize("D,H,KV,window", [(128, 8, 2, 0), (64, 8, 2, 0), (128, 4, 4, 200), (64, 4, 2, 0)])
def test_flash_attention_packed_documents(C, D, H, KV, window):
    """Document-masked flash attention (doc_start / doc_end bounds, tile skipping, boundary masks)
    against the fp32 reference: documents shorter than a tile, spanning several 256-key blocks, and a
    row that is one document."""
    from finetune_controller_amd.ops.attention import _FlashPacked, attention_reference, segments_from_eos

    torch.manual_seed(0)
    B, S = 3, 1024
    ids = _doc_ids(B, S, [[5, 40, 300, 27, 1, 600], [513, 200, 311], [S]])
    seg = segments_from_eos(ids, 2)
    W = (H + 2 * KV) * D
    qkv = bf(torch.randn(B * S, W, device=DEV))
    scale = 1.0 / math.sqrt(D)
    ref_in = qkv.float().clone().requires_grad_(True)
    ref = attention_reference(ref_in, B, S, H, KV, D, True, window, scale, docs=seg)
    x = qkv.clone().requires_grad_(True)
    out = _FlashPacked.apply(x, B, S, H, KV, D, True, window, scale, 0, 0, seg)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    dout = bf(torch.randn(B * S, H * D, device=DEV))
    ref.backward(dout.float())
    out.backward(dout)
    g, gr = x.grad.float(), ref_in.grad
    for lo, hi in ((0, H * D), (H * D, (H + KV) * D), ((H + KV) * D, W)):
        err = (g[:, lo:hi] - gr[:, lo:hi]).abs().max().item()
        mag = gr[:, lo:hi].abs().max().item()
        assert err <= 2e-2 * mag + 2e-2, (lo, err, mag)


def test_llama_packed_documents_hip_matches_documents_alone(C, monkeypatch):
    """Whole model on the HIP path: a packed row's logits equal each document run alone (positions
    restart, attention stays inside the document)."""
    from finetune_controller_amd.models import build_model
    from finetune_controller_amd.models.config import get_config
    from finetune_controller_amd.ops.attention import segments_from_eos

    monkeypatch.setenv("FTC_KERNELS", "hip")
    cfg = get_config("llama-smoke")
    torch.manual_seed(0)
    m = build_model(cfg, None, device=DEV, dtype=torch.bfloat16)
    m.init_weights(seed=3)
    m.eval()
    lens = [256, 100, 156, 512]  # documents of 256 / 512 also run alone on the flash kernels
    ids = torch.randint(3, cfg.vocab_size, (1, sum(lens)), device=DEV)
    ends = torch.tensor(lens).cumsum(0) - 1
    ids[0, ends.to(DEV)] = 2
    seg = segments_from_eos(ids, 2)
    with torch.no_grad():
        packed = m(ids, segments=seg).float()
        lo = 0
        for n in lens:
            alone = m(ids[:, lo:lo + n]).float()
            err = (packed[lo:lo + n] - alone).abs().max().item()
            assert err < 0.05 * alone.abs().max().item() + 0.05, (n, err)
            lo += n


@pytest.mark.parametrize("method", ["lora", "full"])
def test_graph_captured_steps_match_eager(C, tmp_path, method):
    """hipGraph whole-step capture (Trainer graph=True): after the two eager warm-up steps every step
    is one graph replay; losses, grad norms and the parameters follow the eager run under a cosine
    schedule with warmup (device-side lr / bias-correction table)."""
    from finetune_controller_amd.train.trainer import Trainer, TrainConfig

    res = {}
    for graph in (False, True):
        torch.manual_seed(0)
        tr = Trainer(TrainConfig(model="llama-smoke", method=method, batch_size=2, seq_len=256, synthetic=True,
                                 max_steps=7, warmup_steps=3, schedule="cosine", lr=1e-3, graph=graph,
                                 checkpoint_path=str(tmp_path / str(graph)), resume=False, device="cuda",
                                 save_model=False, log_interval=1))
        assert tr.graph_ok() == graph
        last = tr.run()
        res[graph] = (last, tr.opt.param_flat.float().clone(), tr.opt.step_count)
        if graph:
            assert tr._graph is not None and tr._n_graph_calls == 7
        tr.close()
    (le, pe, ce), (lg, pg, cg) = res[False], res[True]
    assert ce == cg == 7
    assert abs(le["loss"] - lg["loss"]) <= 1e-3 * abs(le["loss"]) and abs(le["lr"] - lg["lr"]) < 1e-12
    assert abs(le["grad_norm"] - lg["grad_norm"]) <= 1e-2 * abs(le["grad_norm"]) + 1e-6
    assert (pe - pg).abs().max().item() < 1e-2


@pytest.mark.parametrize("D,H,KV,window", [(128, 32, 8, 0), (128, 8, 8, 0), (64, 32, 8, 0), (128, 64, 8, 0),
                                           (128, 24, 8, 300), (64, 4, 2, 100)])
def test_decode_attention_kernel(C, D, H, KV, window):
    """Split-K decode attention (csrc/kernels/decode_attn.hip) vs the fp32 masked-softmax reference:
    cache lengths inside one chunk, across chunks, at a chunk edge; GQA groups 1..8; sliding window."""
    from finetune_controller_amd.ops.decode import decode_attention_reference

    torch.manual_seed(0)
    B, L = 5, 1100
    q = bf(torch.randn(B, (H + 2 * KV) * D, device=DEV))  # packed qkv row view, q first
    k = bf(torch.randn(B, L, KV * D, device=DEV))
    v = bf(torch.randn(B, L, KV * D, device=DEV))
    lens = torch.tensor([1, 256, 257, 1000, 1100], dtype=torch.int32, device=DEV)
    scale = 1.0 / math.sqrt(D)
    for max_len, B_ in ((1100, B), (1100, 1)):  # the chunk size follows batch x kv heads x length
        k2, v2 = k[:B_].clone(), v[:B_].clone()
        out = C.decode_attention(q[:B_], k2, v2, lens[-B_:].contiguous() if B_ == 1 else lens, H, KV, D, max_len,
                                 scale, window)
        # the kernel appended the current token's K/V (q's k | v columns) at position lens - 1
        ln = lens[-B_:] if B_ == 1 else lens
        rows = torch.arange(B_, device=DEV)
        kr, vr = k[:B_].clone(), v[:B_].clone()
        kr[rows, ln.long() - 1] = q[:B_, H * D:(H + KV) * D]
        vr[rows, ln.long() - 1] = q[:B_, (H + KV) * D:(H + 2 * KV) * D]
        assert torch.equal(k2, kr) and torch.equal(v2, vr)
        ref = decode_attention_reference(q[:B_].float(), kr, vr, ln, H, KV, D, scale, window)
        torch.testing.assert_close(out.float(), ref.float(), atol=2e-2, rtol=2e-2)


def test_kv_cache_decode_logits_match_recompute(C, monkeypatch):
    """Llama on the HIP path: logits of cached decode steps (decode kernel, RoPE at the cache
    position, K/V rows appended per step) equal the last-row logits of re-running the full sequence."""
    from finetune_controller_amd import ops
    from finetune_controller_amd.models import build_model
    from finetune_controller_amd.models.config import get_config

    monkeypatch.setenv("FTC_KERNELS", "hip")
    cfg = get_config("llama-smoke")
    torch.manual_seed(0)
    m = build_model(cfg, None, device=DEV, dtype=torch.bfloat16)
    m.init_weights(seed=2)
    m.eval()
    prompt = torch.randint(3, cfg.vocab_size, (1, 512), device=DEV)
    new = torch.randint(3, cfg.vocab_size, (4,), device=DEV)
    cache = ops.KVCache(len(m.layers), 1, 600, cfg.n_kv_heads, cfg.head_dim, DEV)
    with torch.no_grad():
        cache.row = 0
        m.hidden(prompt, kv_cache=cache)
        cache.finish_prefill(0, 512)
        seq = prompt
        for t in range(4):
            pos = cache.begin_decode()
            x = m.hidden(new[t].view(1, 1), positions=pos, kv_cache=cache)
            cache.end_decode()
            cache.decoding = False
            got = (x @ m.lm_head.t()).float()[-1]
            seq = torch.cat([seq, new[t].view(1, 1)], 1)
            want = m(seq).float()[-1]
            err = (got - want).abs().max().item()
            assert err < 0.03 * want.abs().max().item() + 0.03, (t, err)


def test_generate_hipgraph_matches_eager(C, monkeypatch):
    """Decode steps replayed from a hipGraph produce the same tokens as the eager loop (several
    prompts of different lengths, LoRA adapters live in the augmented GEMMs)."""
    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import get_config
    from finetune_controller_amd.models.generate import generate

    monkeypatch.setenv("FTC_KERNELS", "hip")
    cfg = get_config("llama-smoke")
    torch.manual_seed(0)
    m = build_model(cfg, LoRAConfig(r=16, alpha=32), device=DEV, dtype=torch.bfloat16)
    m.init_weights(seed=2)
    for layer in m.layers:
        for p in layer.lora.values():
            torch.nn.init.normal_(p.B, std=0.02)
    g = torch.Generator().manual_seed(1)
    prompts = [torch.randint(3, cfg.vocab_size, (n,), generator=g).tolist() for n in (7, 300, 64)]
    eager = generate(m, prompts, max_new_tokens=12, graph=False)
    graphed = generate(m, prompts, max_new_tokens=12, graph=True)
    assert eager == graphed and all(len(o) == 12 for o in eager)


def test_accum_mm_fp32_out_bf16_operands(C):
    """fp32 gradient accumulation: bf16 A/B, fp32 C accumulated in place (hipBLASLt out_dtype GEMM)
    against an fp32 reference; repeated accumulation keeps fp32 precision."""
    from finetune_controller_amd.ops.linear import accum_mm

    torch.manual_seed(0)
    out = torch.zeros(384, 512, device=DEV, dtype=torch.float32)
    ref = torch.zeros(384, 512, device=DEV, dtype=torch.float64)
    for _ in range(6):
        a = torch.randn(2048, 384, device=DEV, dtype=torch.bfloat16)
        b = torch.randn(2048, 512, device=DEV, dtype=torch.bfloat16)
        ptr = out.data_ptr()
        accum_mm(out, a.t(), b, 0.5)
        assert out.data_ptr() == ptr and out.dtype == torch.float32
        ref += 0.5 * (a.double().t() @ b.double())
    err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-5, err


def test_full_ft_fp32_grads_hip_match_torch_path(C, monkeypatch):
    """Full fine-tuning with the fp32 gradient buffer and 2 accumulated micro-batches: HIP path vs the
    stock-PyTorch path (same fp32 accumulation semantics), losses and the summed gradient."""
    from finetune_controller_amd.models import build_model
    from finetune_controller_amd.models.config import ModelConfig
    from finetune_controller_amd.train.optim import FlatAdamW

    cfg = ModelConfig("llama", 512, 256, 2, 4, 2, 512, 512, 10000.0, name="llama-test")
    ids = [torch.randint(0, cfg.vocab_size, (2, 256), device=DEV) for _ in range(2)]
    res = {}
    for mode in ("hip", "torch"):
        monkeypatch.setenv("FTC_KERNELS", mode)
        m = build_model(cfg, None, device=DEV, dtype=torch.bfloat16)
        m.init_weights(seed=5)
        opt = FlatAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3, max_grad_norm=1.0,
                        grad_scale=0.5, grad_dtype=torch.float32)
        assert opt.grad_flat.dtype == torch.float32
        opt.zero_grad()
        for x in ids:
            m(x, torch.roll(x, -1, 1)).backward()
        assert all(p.grad is None for p in opt.params)
        res[mode] = opt.grad_flat.clone()
        opt.step()
    gh, gt = res["hip"], res["torch"]
    err = ((gh - gt).norm() / gt.norm()).item()
    assert err < 2e-2, err


def test_copy2d_batched_matches_torch(C):
    """The batched LoRA operand refresh kernel: plain, scaled and transposed strided jobs of mixed sizes
    in one launch equal torch's copy_ / mul (bf16 rounding of the fp32 product)."""
    from finetune_controller_amd.ops import linear as L

    g = torch.Generator(device=DEV).manual_seed(3)
    A = torch.randn(48, 4096, device=DEV, generator=g).to(torch.bfloat16)
    B = torch.randn(6144, 48, device=DEV, generator=g).to(torch.bfloat16)
    big = torch.zeros(6144 + 64, 4096 + 64, device=DEV, dtype=torch.bfloat16)
    bigT = torch.zeros(4096, 6144 + 64, device=DEV, dtype=torch.bfloat16)
    bt = torch.zeros(64, 6144, device=DEV, dtype=torch.bfloat16)
    jobs = [(big[:6144, 4096:4144], B, 1.0), (big[6144:6192, :4096], A, 2.0 / 3.0), (bigT[:, 6144:6192], A.t(), 0.5),
            (bt[:48], B.t(), 1.0)]
    blob = b"".join(L._pack_job(*j) for j in jobs)
    import numpy as np

    table = torch.from_numpy(np.frombuffer(blob, dtype=np.int64).copy()).to(DEV)
    C.copy2d_batched_(table, len(jobs), max(d.numel() for d, _, _ in jobs))
    torch.cuda.synchronize()
    assert torch.equal(big[:6144, 4096:4144], B)
    assert torch.equal(big[6144:6192, :4096], torch.mul(A, 2.0 / 3.0))
    assert torch.equal(bigT[:, 6144:6192], torch.mul(A, 0.5).t())
    assert torch.equal(bt[:48], B.t())
    # nothing outside the job views was written
    assert big[:6144, 4144:].abs().sum() == 0 and big[6192:].abs().sum() == 0 and bt[48:].abs().sum() == 0


def test_batched_refresh_trainer_steps_match_per_projection(C, tmp_path, monkeypatch):
    """LoRA training with the one-launch operand refresh (default) follows the per-projection refresh
    bit for bit over several optimizer steps (A / B change every step)."""
    from finetune_controller_amd.ops import linear as L
    from finetune_controller_amd.train.trainer import Trainer, TrainConfig

    res = {}
    for batched in (True, False):
        monkeypatch.setattr(L, "_BATCH_REFRESH", batched)
        torch.manual_seed(0)
        tr = Trainer(TrainConfig(model="llama-smoke", method="lora", batch_size=2, seq_len=256, synthetic=True,
                                 max_steps=4, warmup_steps=0, lr=1e-2, checkpoint_path=str(tmp_path / str(batched)),
                                 resume=False, device="cuda", save_model=False, log_interval=1))
        last = tr.run()
        res[batched] = (last["loss"], tr.opt.param_flat.float().clone())
        tr.close()
    assert res[True][0] == res[False][0]
    assert torch.equal(res[True][1], res[False][1])


def test_full_ft_overlapped_update_matches_serial(C, monkeypatch, tmp_path):
    """Full fine-tuning through the Trainer with the AdamW update overlapped with the next forward
    (stage-wise on a side stream, FlatAdamW.enable_overlap) vs the serial update: identical losses and
    bitwise-identical parameters / optimizer state after three steps (same kernels, same math)."""
    from finetune_controller_amd.train.trainer import TrainConfig, Trainer

    res = {}
    for ov in ("1", "0"):
        monkeypatch.setenv("FTC_OPT_OVERLAP", ov)
        tc = TrainConfig(model="llama-smoke", method="full", batch_size=2, seq_len=256, synthetic=True, max_steps=3,
                         warmup_steps=0, schedule="constant", lr=1e-3, save_model=False, resume=False, device="cuda",
                         checkpoint_path=str(tmp_path / ov))
        tr = Trainer(tc)
        assert (tr.opt._stages is not None) == (ov == "1")
        losses = [tr.train_step(1e-3).float().item() for _ in range(3)]
        tr.opt.join()
        torch.cuda.synchronize()
        res[ov] = (losses, tr.opt.param_flat.clone(), tr.opt.exp_avg_sq.clone(), tr.opt.grad_flat.clone())
        tr.close()
    (l1, p1, v1, g1), (l0, p0, v0, g0) = res["1"], res["0"]
    assert l1 == l0, (l1, l0)
    assert torch.equal(p1, p0) and torch.equal(v1, v0)
    # the overlapped path zeroes each stage's gradient right after its update; the serial one keeps
    # the last gradients until the next zero_grad
    assert torch.count_nonzero(g1) == 0 and torch.count_nonzero(g0) > 0


@pytest.mark.parametrize("grad_dtype", ["bf16", "fp32"])
def test_full_ft_side_stream_wgrad_matches_serial(C, tmp_path, grad_dtype):
    """Full fine-tuning with every projection's weight gradient on the side stream (ops.linear
    _wgrad_on_side, FTC_DW_STREAM) vs on the main stream: identical losses and bitwise-identical
    parameters, moments and gradients after three steps (same GEMMs, same operands; only the queue
    differs)."""
    from finetune_controller_amd.ops import linear as L
    from finetune_controller_amd.train.trainer import TrainConfig, Trainer

    res = {}
    prior = L.wgrad_stream_active()
    try:
        for side in (True, False):
            L.set_wgrad_stream(side)
            tc = TrainConfig(model="llama-smoke", method="full", batch_size=2, seq_len=256, synthetic=True,
                             max_steps=3, warmup_steps=0, schedule="constant", lr=1e-3, save_model=False,
                             resume=False, device="cuda", grad_dtype=grad_dtype, grad_accum=2,
                             checkpoint_path=str(tmp_path / str(side)))
            tr = Trainer(tc)
            losses = [tr.train_step(1e-3).float().item() for _ in range(3)]
            assert not L._DW_PENDING  # joined by the trainer after every backward
            torch.cuda.synchronize()
            res[side] = (losses, tr.opt.param_flat.clone(), tr.opt.exp_avg_sq.clone(), tr.opt.grad_flat.clone())
            tr.close()
    finally:
        L.set_wgrad_stream(prior)
    (l1, p1, v1, g1), (l0, p0, v0, g0) = res[True], res[False]
    assert l1 == l0, (l1, l0)
    assert torch.equal(g1, g0) and torch.equal(p1, p0) and torch.equal(v1, v0)


@pytest.mark.parametrize("grad_dtype", ["bf16", "fp32"])
def test_full_ft_first_write_grads_match_zeroed(C, tmp_path, grad_dtype):
    """Full fine-tuning with the projection weights' gradient slices left unzeroed and written by a beta = 0
    first GEMM (ops.linear _FIRST_WRITE) vs the zeroed buffer: same losses, gradients and
    parameters over three steps of grad accumulation 2 (the library may pick another GEMM solution for
    beta = 0: equal up to its rounding)."""
    from finetune_controller_amd.ops import linear as L
    from finetune_controller_amd.train.trainer import TrainConfig, Trainer

    res = {}
    prior = L._FIRST_WRITE
    try:
        for fw in (True, False):
            L.set_first_write(fw)
            tc = TrainConfig(model="llama-smoke", method="full", batch_size=2, seq_len=256, synthetic=True,
                             max_steps=3, warmup_steps=0, schedule="constant", lr=1e-3, save_model=False,
                             resume=False, device="cuda", grad_dtype=grad_dtype, grad_accum=2,
                             checkpoint_path=str(tmp_path / str(fw)))
            tr = Trainer(tc)
            losses = [tr.train_step(1e-3).float().item() for _ in range(3)]
            torch.cuda.synchronize()
            L.gradients_final()  # what any reader of the buffer does first (the optimizer step already did)
            res[fw] = (losses, tr.opt.param_flat.float().clone(), tr.opt.grad_flat.float().clone(),
                       sum(1 for p in tr.opt.params if L.is_grad_owned(p)), list(tr.opt.offsets))
            tr.close()
    finally:
        L.set_first_write(prior)
    (l1, p1, g1, owned, offs), (l0, p0, g0, _, _) = res[True], res[False]
    assert owned > 0  # the projection weights were taken off the zeroing pass
    assert max(abs(a - b) / abs(b) for a, b in zip(l1, l0)) < 1e-3, (l1, l0)
    # per parameter slice: a stale or unzeroed slice of one weight cannot hide in a whole-buffer norm
    tol = 1e-4 if grad_dtype == "fp32" else 2e-2
    for o, n in offs:
        a, b = g1[o:o + n], g0[o:o + n]
        assert ((a - b).norm() / b.norm().clamp_min(1e-30)).item() < tol, (o, n)
    assert ((p1 - p0).norm() / p0.norm()).item() < 1e-4


@pytest.mark.parametrize("method", ["full", "lora"])
def test_gpt2_steps_hip_match_torch_path(C, monkeypatch, method):
    """GPT-2 geometry (d 768, 12 heads of 64, odd vocab 50257, tied lm_head, LayerNorm/GELU, learned
    positions) on the HIP path -- D=64 flash attention, chunked CE over the odd vocabulary, flat AdamW
    (+ LoRA on the packed projections) -- against the stock-PyTorch path over three steps."""
    from finetune_controller_amd.models import LoRAConfig, build_model
    from finetune_controller_amd.models.config import ModelConfig
    from finetune_controller_amd.train.optim import FlatAdamW

    cfg = ModelConfig("gpt2", 50257, 768, 2, 12, 12, 3072, 1024, tie_embeddings=True, name="gpt2-2l")
    lc = LoRAConfig(r=16, alpha=32) if method == "lora" else None
    ids = torch.randint(0, cfg.vocab_size, (2, 512), device=DEV)
    labels = torch.roll(ids, -1, 1)
    res = {}
    for mode in ("hip", "torch"):
        monkeypatch.setenv("FTC_KERNELS", mode)
        torch.manual_seed(0)
        m = build_model(cfg, lc, device=DEV, dtype=torch.bfloat16)
        m.init_weights(seed=5)
        if lc is not None:
            m.freeze_base()
        opt = FlatAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-3 if lc else 1e-4, max_grad_norm=1.0)
        losses = []
        for _ in range(3):
            opt.zero_grad()
            loss = m(ids, labels)
            loss.backward()
            opt.step()
            losses.append(loss.float().item())
        res[mode] = (losses, opt.param_flat.float().clone())
    (lh, ph), (lt, pt) = res["hip"], res["torch"]
    for a, b in zip(lh, lt):
        assert abs(a - b) < 2e-2 * abs(b), (lh, lt)
    assert lh[2] < lh[0]
    assert (ph - pt).abs().max().item() < 1e-2
