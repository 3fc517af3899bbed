#!/usr/bin/env python3
"""SwiGLU + LoRA tail products at the Llama-3-8B MLP shape (T = 16384, F = 14336, Rp = 64):
fused kernels (csrc/kernels/swiglu_lora.hip) against the plain SwiGLU kernel + a skinny hipBLASLt GEMM
that re-reads the produced tensor.  Prints one JSON line per variant (ms, effective HBM TB/s)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    import finetune_controller_amd._C as C

    T, F, Rp = int(os.environ.get("T", 16384)), 14336, 64
    bf = torch.bfloat16
    gu = torch.randn(T, 2 * F, device="cuda", dtype=bf)
    da = torch.randn(T, F, device="cuda", dtype=bf)
    am = torch.zeros(Rp, F, device="cuda", dtype=bf)
    am[:16] = 0.1 * torch.randn(16, F, device="cuda", dtype=bf)
    bt = torch.zeros(Rp, 2 * F, device="cuda", dtype=bf)
    bt[:32] = 0.1 * torch.randn(32, 2 * F, device="cuda", dtype=bf)
    bt[:16, F:] = 0  # block-diagonal B of the packed gate|up projection (r = 16 per segment)
    bt[16:32, :F] = 0
    B = bt.t().contiguous()  # [2F, Rp] like big[:N, K:]
    res = {}

    def fwd_plain():
        a = C.swiglu_fwd(gu, Rp)
        full = a.as_strided((T, F + Rp), (F + Rp, 1))
        torch.mm(a, am.t(), out=full[:, F:])

    def bwd_plain():
        d = C.swiglu_bwd(da, gu, Rp)
        full = d.as_strided((T, 2 * F + Rp), (2 * F + Rp, 1))
        torch.mm(d, B, out=full[:, 2 * F:])

    xa = torch.randn(T, 4160, device="cuda", dtype=bf)[:, 4096:4128]
    dyb = torch.randn(T, 4160, device="cuda", dtype=bf)[:, 4096:4112]
    mgB = torch.zeros(2 * F, 32, device="cuda", dtype=bf)
    mgA = torch.zeros(16, F, device="cuda", dtype=bf)
    h = torch.randn(T, F + Rp, device="cuda", dtype=bf)[:, :F]

    def bwd_split_wgrad():
        d = C.swiglu_bwd_lora(da, gu, Rp, bt, 2, True)
        C.lora_wgrad_(mgB, d, xa, 16, 1.0, 1.0, [F, 2 * F], [0, 16], [0, 16])
        C.lora_wgrad_(mgA.t(), h, dyb, 16, 0.5, 1.0)

    variants = {
        "fwd_swiglu_only": lambda: C.swiglu_fwd(gu, Rp),
        "fwd_plain+gemm": fwd_plain,
        "fwd_fused_nct1": lambda: C.swiglu_fwd_lora(gu, Rp, am, 1),
        "bwd_swiglu_only": lambda: C.swiglu_bwd(da, gu, Rp),
        "bwd_plain+gemm": bwd_plain,
        "bwd_fused_nct2": lambda: C.swiglu_bwd_lora(da, gu, Rp, bt, 2, False),
        "bwd_fused_nct2_split": lambda: C.swiglu_bwd_lora(da, gu, Rp, bt, 2, True),
        "bwd_split+lora_wgrad_dB_gu_dA_down": bwd_split_wgrad,
        "bwd_fused_wgrad": lambda: C.swiglu_bwd_wgrad(da, gu, Rp, bt, xa, dyb, mgB, mgA, 1.0, 0.5),
    }
    for name, fn in variants.items():
        ms = timeit(fn)
        nbytes = (T * 2 * F * 2 + T * F * 2) if name.startswith("fwd") else (T * 2 * F * 2 * 2 + T * F * 2)
        res[name] = ms
        print(json.dumps({"variant": name, "ms": round(ms, 4), "min_bytes_TBps": round(nbytes / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
