#!/usr/bin/env python3
"""Weight-gradient GEMM dW[N,K] (+)= dy^T x at the Llama-3-8B full-FT shapes (T = 16384): variants of
operand presentation for hipBLASLt.  One JSON line per shape."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.bench_gemms import timeit  # noqa: E402

T = 16384
bf = torch.bfloat16
for name, (K, N) in {"qkv": (4096, 6144), "o": (4096, 4096), "gu": (4096, 28672), "down": (14336, 4096)}.items():
    x = torch.randn(T, K, device="cuda", dtype=bf)
    dy = torch.randn(T, N, device="cuda", dtype=bf)
    mg = torch.zeros(N, K, device="cuda", dtype=bf)
    mgf = torch.zeros(N, K, device="cuda", dtype=torch.float32)
    mgT = torch.zeros(K, N, device="cuda", dtype=bf)
    fl = 2 * T * N * K
    r = {"gemm": name}
    r["addmm_bf16"] = timeit(lambda: mg.addmm_(dy.t(), x))
    r["mm_bf16"] = timeit(lambda: torch.mm(dy.t(), x, out=mg))
    r["addmm_T_bf16"] = timeit(lambda: mgT.addmm_(x.t(), dy))
    try:
        r["mm_f32out"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
    except Exception as e:  # noqa: BLE001
        r["mm_f32out"] = str(e)[:60]
    dyT = dy.t().contiguous()
    xT = x.t().contiguous()
    r["transpose_dy"] = timeit(lambda: dyT.copy_(dy.t()))
    r["mm_dyT_x"] = timeit(lambda: torch.mm(dyT, x, out=mg))
    r["mm_dyT_xT"] = timeit(lambda: torch.mm(dyT, xT.t(), out=mg))
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()} |
                     {"best_tflops": round(fl / min(v for k2, v in r.items() if isinstance(v, float) and k2 != "transpose_dy") / 1e9)}), flush=True)
    del x, dy, mg, mgf, mgT, dyT, xT
