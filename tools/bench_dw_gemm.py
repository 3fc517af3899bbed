#!/usr/bin/env python3
"""Weight-gradient GEMM dW[N, K] += dy^T x (reduction over T = 16384 tokens) at the Llama-3-8B full
fine-tune shapes, in every operand layout hipBLASLt can be handed:

  tt  : addmm_(dy.t(), x)           dy [T, N], x [T, K] row-major (what autograd produces)
  tr  : dW^T += x^T dy  into a [K, N] buffer
  nt  : addmm_(dyT, x)              dyT [N, T] contiguous
  tn  : addmm_(dy.t(), xT.t())      xT  [K, T] contiguous
  nn  : addmm_(dyT, xT.t())         both transposed
Prints ms and TFLOP/s per variant plus the cost of producing a transposed copy."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.bench_gemms import timeit  # noqa: E402


def main():
    T = 16384
    bf = torch.bfloat16
    for name, (N, K) in {"qkv": (6144, 4096), "o": (4096, 4096), "gu": (28672, 4096), "down": (4096, 14336),
                         "lm_head": (128256, 4096)}.items():
        Tn = 4096 if name == "lm_head" else T  # lm_head dW is accumulated per CE chunk
        dy = torch.randn(Tn, N, device="cuda", dtype=bf)
        x = torch.randn(Tn, K, device="cuda", dtype=bf)
        dW = torch.zeros(N, K, device="cuda", dtype=bf)
        dWt = torch.zeros(K, N, device="cuda", dtype=bf)
        dyT = dy.t().contiguous()
        xT = x.t().contiguous()
        fl = 2 * Tn * N * K
        res = {"gemm": name}
        for v, fn in (("tt", lambda: dW.addmm_(dy.t(), x)), ("tr", lambda: dWt.addmm_(x.t(), dy)),
                      ("nt", lambda: dW.addmm_(dyT, x)), ("tn", lambda: dW.addmm_(dy.t(), xT.t())),
                      ("nn", lambda: dW.addmm_(dyT, xT.t()))):
            ms = timeit(fn, iters=10)
            res[v] = [round(ms, 3), round(fl / ms / 1e9)]
        res["transpose_dy_ms"] = round(timeit(lambda: dy.t().contiguous(), iters=10), 3)
        res["transpose_x_ms"] = round(timeit(lambda: x.t().contiguous(), iters=10), 3)
        print(json.dumps(res), flush=True)
        del dy, x, dW, dWt, dyT, xT


if __name__ == "__main__":
    main()
