#!/usr/bin/env python3
"""hipBLASLt GEMM efficiency at the exact Llama-3-8B LoRA step shapes (T = 16384 tokens):
forward  y = X_aug W_aug^T   (K + 64 augmented columns)   and   backward dx = [dy | dyB] [W ; sA].
Prints TFLOP/s per shape; compares the augmented K/N against the plain one."""
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
    T = 16384
    bf = torch.bfloat16
    shapes = {"qkv": (4096, 6144), "o": (4096, 4096), "gu": (4096, 28672), "down": (14336, 4096), "lm_head": (4096, 128256)}
    tot_ms = 0.0
    for name, (K, N) in shapes.items():
        for aug in (0, 64):
            if name == "lm_head" and aug:
                continue
            x = torch.randn(T, K + aug, device="cuda", dtype=bf)
            W = torch.randn(N, K + aug, device="cuda", dtype=bf)
            dy = torch.randn(T, N + aug, device="cuda", dtype=bf)
            W2 = torch.randn(N + aug, K, device="cuda", dtype=bf)
            f = timeit(lambda: x @ W.t())
            b = timeit(lambda: dy @ W2)
            fl = 2 * T * N * K
            if aug or name == "lm_head":
                tot_ms += f + b
            print(json.dumps({"gemm": name, "aug": aug, "fwd_ms": round(f, 3), "fwd_tflops": round(fl / f / 1e9, 1),
                              "bwd_dx_ms": round(b, 3), "bwd_tflops": round(fl / b / 1e9, 1)}), flush=True)
            del x, W, dy, W2
    print(json.dumps({"per_layer_plus_head_ms": round(tot_ms, 2)}))


if __name__ == "__main__":
    main()
