#!/usr/bin/env python3
"""How the augmented GEMMs' extra K (forward) / N (backward, TN layout) columns and the operand row
stride affect hipBLASLt at the Llama-3-8B LoRA step shapes (T = 16384).

Forward  y[T, N]  = X[:, :K'] W[:, :K']^T   with K' = K + aug, X / W row stride ld >= K'
Backward dx[T, K] = dY[:, :N'] Wt[:, :N']^T with N' = N + aug (Wt = [W ; sA]^T stored K x ld)
Prints one JSON line per (shape, aug, ld): ms and model TFLOP/s (2 T N K, the un-augmented work)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.bench_gemms import timeit  # noqa: E402


def main():
    T = 16384
    bf = torch.bfloat16
    shapes = {"qkv": (4096, 6144), "o": (4096, 4096), "gu": (4096, 28672), "down": (14336, 4096)}
    for name, (K, N) in shapes.items():
        fl = 2 * T * N * K
        for aug, pad in ((0, 0), (64, 0), (64, 64), (16, 0), (32, 0), (128, 0)):
            Kp, ld = K + aug, K + aug + pad
            x = torch.randn(T, ld, device="cuda", dtype=bf)
            w = torch.randn(N, ld, device="cuda", dtype=bf)
            f = timeit(lambda: torch.mm(x[:, :Kp], w[:, :Kp].t()))
            Np, ldn = N + aug, N + aug + pad
            dy = torch.randn(T, ldn, device="cuda", dtype=bf)
            wt = torch.randn(K, ldn, device="cuda", dtype=bf)
            b = timeit(lambda: torch.mm(dy[:, :Np], wt[:, :Np].t()))
            print(json.dumps({"gemm": name, "aug": aug, "ld_pad": pad, "fwd_ms": round(f, 3),
                              "fwd_tf": round(fl / f / 1e9), "bwd_ms": round(b, 3), "bwd_tf": round(fl / b / 1e9)}),
                  flush=True)
            del x, w, dy, wt


if __name__ == "__main__":
    main()
