#!/usr/bin/env python3
"""NF4 GEMM microbenchmark (K8): fused NF4-dequant MFMA kernel vs dequantise + hipBLASLt vs a plain
bf16 GEMM, at Mistral-7B projection shapes, M = activation rows.  Prints one JSON line per shape.
Sets the crossover ``ops/nf4.py: FUSED_MAX_ROWS``."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from finetune_controller_amd.ops import nf4  # noqa: E402
from finetune_controller_amd.ops._backend import ext  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters * 1e3  # us


def main():
    C = ext()
    for N, K in ((4096, 4096), (28672, 4096), (4096, 14336)):
        W = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
        qw = nf4.NF4Weight.quantize(W)
        for M in (1, 16, 64, 128, 256, 512, 1024):
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            fused = timeit(lambda: C.nf4_linear(x, qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, N,
                                                qw.block, qw.block2))
            deq = timeit(lambda: x @ qw.dequantize().t())
            bf = timeit(lambda: x @ W.t())
            wbytes = qw.nbytes()
            print(json.dumps({"N": N, "K": K, "M": M, "fused_us": round(fused, 1), "dequant_gemm_us": round(deq, 1),
                              "bf16_gemm_us": round(bf, 1), "fused_weight_GBps": round(wbytes / fused / 1e3, 1),
                              "fused_tflops": round(2 * M * N * K / fused / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
