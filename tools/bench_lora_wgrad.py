#!/usr/bin/env python3
"""LoRA weight-gradient GEMMs of one Llama-3-8B all-linear r16 layer (T = 16384): hipBLASLt beta=1
addmm_ vs csrc/kernels/lora_wgrad.hip.  One JSON line per GEMM (us and effective TB/s of X)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from finetune_controller_amd.ops._backend import load_ext  # noqa: E402
from tools.bench_gemms import timeit  # noqa: E402

C = load_ext(required=True)
T = 16384
bf = torch.bfloat16
# (name, M, Xwidth(buffer cols), R): dB per block (packed qkv: q/k/v, gu: gate/up), dA of each projection
cases = [("dB_q", 4096, 6144 + 64, 16), ("dB_kv", 1024, 6144 + 64, 16), ("dB_o", 4096, 4096 + 64, 16),
         ("dB_gate", 14336, 28672 + 64, 16), ("dB_down", 4096, 4096 + 64, 16),
         ("dA_qkv", 4096, 4096 + 64, 48), ("dA_o", 4096, 4096 + 64, 16), ("dA_gu", 4096, 4096 + 64, 32),
         ("dA_down", 14336, 14336 + 64, 16)]
tot = [0.0, 0.0]
for name, M, W, R in cases:
    Xb = torch.randn(T, W, device="cuda", dtype=bf)
    X = Xb[:, :M]
    Y = Xb[:, W - 64:W - 64 + R]
    out = torch.zeros(M, R, device="cuda", dtype=bf)
    t_blas = timeit(lambda: out.addmm_(X.t(), Y))
    t_hip = timeit(lambda: C.lora_wgrad_(out, X, Y, R, 1.0, 1.0))
    mult = 2 if name in ("dB_kv", "dB_gate") else 1  # k and v / gate and up
    tot[0] += mult * t_blas
    tot[1] += mult * t_hip
    gb = T * M * 2 / 1e9
    print(json.dumps({"gemm": name, "M": M, "R": R, "hipblaslt_us": round(t_blas * 1e3, 1),
                      "hip_us": round(t_hip * 1e3, 1), "hip_TBps": round(gb / t_hip, 2)}), flush=True)
    del Xb
print(json.dumps({"per_layer_us": {"hipblaslt": round(tot[0] * 1e3, 1), "hip": round(tot[1] * 1e3, 1)}}))
# packed projections in one launch (segments): dB of q|k|v and of gate|up
for name, N, segs, Rt in (("dB_qkv_1launch", 6144, [(4096, 0), (5120, 16), (6144, 32)], 48),
                          ("dB_gu_1launch", 28672, [(14336, 0), (28672, 16)], 32)):
    Xb = torch.randn(T, N + 64, device="cuda", dtype=bf)
    X, Y = Xb[:, :N], Xb[:, N:N + 64]
    out = torch.zeros(N, Rt, device="cuda", dtype=bf)
    t = timeit(lambda: C.lora_wgrad_(out, X, Y, 16, 1.0, 1.0, [a for a, _ in segs], [c for _, c in segs],
                                     [c for _, c in segs]))
    print(json.dumps({"gemm": name, "hip_us": round(t * 1e3, 1), "hip_TBps": round(T * N * 2 / 1e9 / t, 2)}))
    del Xb
