"""LAB-ONLY: the hand-written projection (NT, RoPE epilogue) and weight-gradient (TN) GEMMs.

They left ``_C.so`` in round 6 (VERDICT r5 Next #4: ship only winners -- neither beats hipBLASLt on a shipped
shape) and live in ``tools/gemm_lab/`` (``libgemm_lab.so``, ctypes front-end ``tools/gemm_lab/lab.py``).
These numerics tests stay as the lab's regression suite; they run only with ``FTC_LAB=1`` on a GPU box
after ``bash tools/gemm_lab/build.sh``:

    FTC_LAB=1 python -m pytest tests/test_gemm_lab.py -m gpu
"""
import os
import sys

import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.lab,
              pytest.mark.skipif(os.environ.get("FTC_LAB") != "1", reason="lab-only (FTC_LAB=1)")]

DEV = "cuda"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lab():
    sys.path.insert(0, ROOT)
    from tools.gemm_lab.lab import load

    return load()


@pytest.mark.parametrize("cdtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K,lda_pad,beta", [(256, 256, 64, 0, 0.0), (512, 768, 1024, 0, 1.0),
                                                (768, 256, 4096, 64, 1.0), (2048, 1024, 192, 0, 0.5)])
def test_gemm_tn(lab, cdtype, M, N, K, lda_pad, beta):
    """Weight-gradient GEMM c = beta c + alpha a^T b (a [K, M], b [K, N] as stored) vs an fp32 reference;
    lda_pad: a is a column view of a wider buffer (the LoRA-padded activation rows)."""
    torch.manual_seed(2)
    abuf = (torch.rand(K, M + lda_pad, device=DEV) * 2 - 1).to(torch.bfloat16)
    a = abuf[:, :M]
    b = (torch.rand(K, N, device=DEV) * 2 - 1).to(torch.bfloat16)
    c = torch.randn(M, N, device=DEV).to(cdtype)
    ref = beta * c.float() + 0.5 * (a.float().t() @ b.float())
    assert lab.gemm_tn_ok(c, a, b)
    lab.gemm_tn_(c, a, b, 0.5, beta)
    tol = 2e-2 * (K ** 0.5) / 8 if cdtype == torch.bfloat16 else 1e-3 * (K ** 0.5) / 8
    torch.testing.assert_close(c.float(), ref, atol=tol, rtol=1e-2 if cdtype == torch.bfloat16 else 1e-4)


def test_gemm_tn_rejects(lab):
    a = torch.zeros(64, 200, device=DEV, dtype=torch.bfloat16)  # M not a multiple of 256
    b = torch.zeros(64, 256, device=DEV, dtype=torch.bfloat16)
    c = torch.zeros(200, 256, device=DEV, dtype=torch.bfloat16)
    assert not lab.gemm_tn_ok(c, a, b)
    with pytest.raises(RuntimeError):
        lab.gemm_tn_(c, a, b, 1.0, 0.0)


@pytest.mark.parametrize("cdtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,N,K,pad,beta", [(256, 256, 64, 0, 0.0), (512, 768, 4160, 64, 0.0), (768, 512, 128, 8, 1.0),
                                            (256, 1024, 1088, 0, -0.5), (512, 256, 192, 0, 0.0)])
def test_gemm_nt(lab, cdtype, M, N, K, pad, beta):
    """Projection GEMM c = alpha a b^T + beta c (a [M, K], b [N, K] K-contiguous, a a column view of a wider
    row buffer when pad > 0) vs an fp32 reference; asymmetric integer-valued operands first (exact
    in fp32: any fragment / output permutation error shows as a wrong integer), then random data."""
    torch.manual_seed(3)
    abuf = torch.randint(-3, 4, (M, K + pad), device=DEV).to(torch.bfloat16)
    a = abuf[:, :K]
    b = (torch.arange(N * K, device=DEV).reshape(N, K) % 7 - 3).to(torch.bfloat16)
    c = torch.zeros(M, N, device=DEV, dtype=cdtype)
    assert lab.gemm_nt_ok(c, a, b)
    lab.gemm_nt_(c, a, b, 1.0, 0.0)
    exact = a.double() @ b.double().t()  # integer sums < 2^24: exact in the fp32 accumulator, one rounding
    assert torch.equal(c, exact.to(cdtype))
    abuf = (torch.rand(M, K + pad, device=DEV) * 2 - 1).to(torch.bfloat16)
    a = abuf[:, :K]
    b = (torch.rand(N, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    c = torch.randn(M, N, device=DEV).to(cdtype)
    ref = beta * c.float() + 0.5 * (a.float() @ b.float().t())
    lab.gemm_nt_(c, a, b, 0.5, beta)
    tol = 2e-2 * (K ** 0.5) / 8 if cdtype == torch.bfloat16 else 1e-3 * (K ** 0.5) / 8
    torch.testing.assert_close(c.float(), ref, atol=tol, rtol=1e-2 if cdtype == torch.bfloat16 else 1e-4)


@pytest.fixture
def nt_config(lab):
    """Restores the projection GEMM's default launch configuration after a test that changes it."""
    yield lab
    lab.gemm_nt_config(0, -8, 32)


@pytest.mark.parametrize("cfg", [(1, 1, 1), (3, 4, 1), (8, -2, 1), (16, 2, 2), (5, -16, 1), (4, -8, 1), (0, -8, 32)])
@pytest.mark.parametrize("M,N,K", [(1024, 768, 64), (768, 1280, 128), (512, 1024, 448)])
def test_gemm_nt_persistent(nt_config, cfg, M, N, K):
    """The persistent grid walks several tiles per workgroup (grid capped below the tile count) with the
    super-stage stream running across tile boundaries -- including K = 64 (one stage per tile: the next
    tile's first stage is prefetched while the current one is still being read) -- under every tile
    order: exact integer products, every tile checked."""
    lab = nt_config
    lab.gemm_nt_config(*cfg)
    torch.manual_seed(11)
    a = torch.randint(-3, 4, (M, K), device=DEV).to(torch.bfloat16)
    b = (torch.arange(N * K, device=DEV).reshape(N, K) % 5 - 2).to(torch.bfloat16)
    c = torch.full((M, N), 7.0, device=DEV, dtype=torch.bfloat16)
    lab.gemm_nt_(c, a, b, 1.0, 0.0)
    assert torch.equal(c, (a.double() @ b.double().t()).to(torch.bfloat16))
    cf = torch.zeros(M, N, device=DEV, dtype=torch.float32)
    lab.gemm_nt_(cf, a, b, 1.0, 0.0)
    assert torch.equal(cf, (a.double() @ b.double().t()).float())


@pytest.mark.parametrize("name,K,N", [("qkv_fwd", 4096 + 64, 6144), ("down_dx", 4096 + 64, 14336)])
def test_gemm_nt_production_shape(lab, name, K, N):
    """The headline step's shapes (T = 4 x 4096 tokens, LoRA-augmented K): bit-identical to torch.mm
    (hipBLASLt accumulates the same 16x16x32 MFMA chain in K order) and close to an fp32 reference on a
    row sample spread over every M tile."""
    torch.manual_seed(12)
    M = 16384
    a = torch.empty(M, K, device=DEV, dtype=torch.bfloat16).uniform_(-1, 1)
    b = torch.empty(N, K, device=DEV, dtype=torch.bfloat16).uniform_(-1, 1)
    c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    lab.gemm_nt_(c, a, b, 1.0, 0.0)
    lib = torch.mm(a, b.t())
    rows = torch.arange(0, M, 97, device=DEV)
    ref = a[rows].float() @ b.float().t()
    torch.testing.assert_close(c[rows].float(), ref, atol=3e-2 * (K ** 0.5) / 8, rtol=1e-2)
    assert torch.equal(c, lib), f"{name}: {(c.float() - lib.float()).abs().max().item()} max |ours - torch.mm|"


@pytest.mark.parametrize("with_pos", [False, True])
def test_gemm_nt_rope_epilogue(lab, with_pos):
    """qkv projection with RoPE fused into the GEMM epilogue (head_dim 128, q and k heads rotated, v not)
    vs the fp32 product rotated by the reference RoPE."""
    from finetune_controller_amd.ops.rope import RotaryTable, _rope_ref

    torch.manual_seed(5)
    H, KV, D, S = 4, 2, 128, 256
    M, K = 512, 320
    N = (H + 2 * KV) * D
    a = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    w = (torch.rand(N, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    tab = RotaryTable(D, 1024, 500000.0)
    cos, sin = tab.get(DEV)
    pos = (torch.arange(M, device=DEV, dtype=torch.int32) * 7 % 1000) if with_pos else None
    c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    lab.gemm_nt_rope_(c, a, w, cos, sin, pos, S, H + KV)
    ref = _rope_ref((a.float() @ w.float().t()), cos, sin, H + KV, D, S, pos, False)
    tol = 2e-2 * (K ** 0.5) / 8
    torch.testing.assert_close(c.float(), ref, atol=tol, rtol=1e-2)


def test_gemm_nt_rejects(lab):
    a = torch.zeros(256, 40, device=DEV, dtype=torch.bfloat16)  # K not a multiple of 32
    b = torch.zeros(256, 40, device=DEV, dtype=torch.bfloat16)
    c = torch.zeros(256, 256, device=DEV, dtype=torch.bfloat16)
    assert not lab.gemm_nt_ok(c, a, b)
    with pytest.raises(RuntimeError):
        lab.gemm_nt_(c, a, b, 1.0, 0.0)
    assert not lab.gemm_nt_ok(c[:, :200], a, b[:200])  # N not a multiple of 256
