#!/usr/bin/env python3
"""The base GEMMs of one Llama-3-8B LoRA step, one shape at a time, for counter collection.

Every GEMM of the flagship step is ``C[T, n] = A[T, k] . B[n, k]^T`` on hipBLASLt (the augmented
LoRA forms of ops/linear.py: forward ``[x | s x A^T] . [W | B]^T`` with k = K + 64, backward
``[dy | dy B] . [W ; s A]`` through the transposed frozen-weight copy with k = N + 64).  T = 16384
tokens (micro-batch 4 x 4096).  Between shapes a fill kernel whose element count encodes the
shape index marks the boundary (``tools/pmc_md.py --labels`` splits the dispatches there; marker
traces cannot be combined with ``--pmc`` on this pool).  Writes the ordered labels + FLOPs to
``--labels`` and prints one timing line per shape (outside the profiler the same numbers are a
plain benchmark).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

T = 16384
SHAPES = [  # (label, k, n)
    ("qkv fwd", 4096 + 64, 6144), ("o fwd", 4096 + 64, 4096), ("gu fwd", 4096 + 64, 28672),
    ("down fwd", 14336 + 64, 4096), ("down bwd dx", 4096 + 64, 14336), ("gu bwd dx", 28672 + 64, 4096),
    ("o bwd dx", 4096 + 64, 4096), ("qkv bwd dx", 6144 + 64, 4096), ("lm_head fwd", 4096, 128256),
]
SENTINEL_BASE = 1 << 20  # fill of SENTINEL_BASE + i elements marks the start of shape i


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--labels", default="gpurun_out/pmc_gemm_labels.json")
    ap.add_argument("--ours", action="store_true",
                    help="also run the lab NT GEMM (tools/gemm_lab/gemm_nt.hip, libgemm_lab.so) on every shape, after the "
                         "library: its own kernel row in the counter table")
    a = ap.parse_args()
    C = None
    if a.ours:
        from tools.gemm_lab.lab import load

        C = load()
    bf = torch.bfloat16
    torch.manual_seed(0)
    labels = []
    for i, (name, k, n) in enumerate(SHAPES):
        x = torch.empty(T, k, device="cuda", dtype=bf).uniform_(-1, 1)  # random data: DVFS (guide §5.4 r25)
        w = torch.empty(n, k, device="cuda", dtype=bf).uniform_(-1, 1)
        y = torch.empty(T, n, device="cuda", dtype=bf)
        torch.empty(SENTINEL_BASE + i, device="cuda", dtype=torch.uint8).fill_(1)  # shape i starts here
        torch.matmul(x, w.t(), out=y)  # warm-up (same kernel; counted with the shape)
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(a.iters):
            torch.matmul(x, w.t(), out=y)
        en.record()
        torch.cuda.synchronize()
        ms = st.elapsed_time(en) / a.iters
        if C is not None and C.gemm_nt_ok(y, x, w):
            C.gemm_nt_(y, x, w, 1.0, 0.0)
            torch.cuda.synchronize()
            st.record()
            for _ in range(a.iters):
                C.gemm_nt_(y, x, w, 1.0, 0.0)
            en.record()
            torch.cuda.synchronize()
            mo = st.elapsed_time(en) / a.iters
            print(json.dumps({"gemm": name, "kernel": "ours", "ms": round(mo, 3),
                              "tflops": round(2.0 * T * n * k / mo / 1e9, 1)}), flush=True)
        fl = 2.0 * T * n * (k - 64 if k % 256 == 64 else k)  # model FLOPs exclude the LoRA pad columns
        labels.append({"label": name, "M": T, "N": n, "K": k, "flops": 2.0 * T * n * k, "model_flops": fl})
        print(json.dumps({"gemm": name, "M": T, "N": n, "K": k, "ms": round(ms, 3),
                          "tflops": round(2.0 * T * n * k / ms / 1e9, 1)}), flush=True)
        del x, w, y
    os.makedirs(os.path.dirname(a.labels) or ".", exist_ok=True)
    with open(a.labels, "w") as f:
        json.dump({"sentinel_base": SENTINEL_BASE, "shapes": labels}, f)


if __name__ == "__main__":
    main()
