#!/usr/bin/env python3
"""RMSNorm (+residual) forward / backward kernels at the Llama-3-8B shape (16384 x 4096, bf16):
ms and effective HBM TB/s (bytes a streaming kernel must move)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tools.bench_gemms import timeit  # noqa: E402


def main():
    import finetune_controller_amd._C as C

    T, d = 16384, 4096
    bf = torch.bfloat16
    x = torch.randn(T, d, device="cuda", dtype=bf)
    r = torch.randn(T, d, device="cuda", dtype=bf)
    w = torch.rand(d, device="cuda", dtype=bf) + 0.5
    y, rstd, h = C.rmsnorm_fwd(x, r, w, 1e-5)
    dy = torch.randn(T, d, device="cuda", dtype=bf)
    dres = torch.randn(T, d + 64, device="cuda", dtype=bf)[:, :d]
    nb = T * d * 2
    xt = torch.randn(T, d + 64, device="cuda", dtype=bf)
    bm = torch.zeros(64, d, device="cuda", dtype=bf)
    bm[:48] = 0.05 * torch.randn(48, d, device="cuda", dtype=bf)
    for nct in (1, 3):
        ms = timeit(lambda: C.tail_gemm_(xt[:, :d], bm, nct, 64))
        ms2 = timeit(lambda: torch.mm(xt[:, :d], bm.t(), out=torch.empty(T, 64, device="cuda", dtype=bf)))
        print(json.dumps({"kernel": f"tail_gemm_nct{nct}", "ms": round(ms, 4), "TBps": round(nb / ms / 1e9, 2),
                          "hipblaslt_ms": round(ms2, 4)}), flush=True)
    for name, fn, nbytes in (("fwd_res", lambda: C.rmsnorm_fwd(x, r, w, 1e-5, 64), 4 * nb),
                             ("bwd_dres_frozen", lambda: C.rmsnorm_bwd(dy, h, w, rstd, dres, False, 64), 4 * nb),
                             ("bwd_dres_dw", lambda: C.rmsnorm_bwd(dy, h, w, rstd, dres, True, 64), 4 * nb)):
        ms = timeit(fn)
        print(json.dumps({"kernel": name, "ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
