#!/usr/bin/env python3
"""Element-wise stream kernels at the Llama-3-8B step shapes (T = 16384): plain SwiGLU fwd / bwd (full FT),
RoPE over q|k, the split-K fold of the down-projection weight gradient, NF4 row dequant (QLoRA forward
operand).  One JSON line per op (best-of-rounds ms, effective TB/s); run once per grid policy."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, iters=20, rounds=3):
    best = 1e30
    for _ in range(rounds):
        fn()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(iters):
            fn()
        en.record()
        torch.cuda.synchronize()
        best = min(best, st.elapsed_time(en) / iters)
    return best


def main():
    import finetune_controller_amd._C as C  # noqa: F401
    from finetune_controller_amd.ops import nf4 as N

    T, F, d = 16384, 14336, 4096
    bf = torch.bfloat16
    dev = "cuda"
    tag = os.environ.get("TAG", "")
    gu = torch.randn(T, 2 * F, device=dev, dtype=bf)
    da = torch.randn(T, F, device=dev, dtype=bf)
    ops = {
        "swiglu_fwd": (lambda: C.swiglu_fwd(gu, 0), T * 2 * F * 2 + T * F * 2),
        "swiglu_bwd": (lambda: C.swiglu_bwd(da, gu, 0), T * 2 * F * 2 + T * F * 2 + T * 2 * F * 2),
    }
    parts = torch.randn(2, d, F, device=dev)
    dw = torch.empty(d, F, device=dev, dtype=bf)
    ops["splitk_sum_down_dw"] = (lambda: C.splitk_sum_(dw, parts, 0.0), 2 * d * F * 4 + d * F * 2)
    res = {}
    for name, (fn, nbytes) in ops.items():
        ms = timeit(fn)
        res[name] = ms
        print(json.dumps({"op": name, "tag": tag, "ms": round(ms, 4), "TBps": round(nbytes / ms / 1e9, 3)}), flush=True)
    del gu, da, parts, dw
    w = torch.randn(F, d, device=dev, dtype=bf)
    qw = N.NF4Weight.quantize(w)
    out = torch.empty(F, d, device=dev, dtype=bf)
    ms = timeit(lambda: N._dequant_into(qw, out, False))
    print(json.dumps({"op": "nf4_dequant_rows", "tag": tag, "ms": round(ms, 4),
                      "TBps": round((F * d // 2 + F * d * 2) / ms / 1e9, 3)}), flush=True)
    outT = torch.empty(d, F, device=dev, dtype=bf)
    ms = timeit(lambda: N._dequant_into(qw, outT, True))
    print(json.dumps({"op": "nf4_dequant_t", "tag": tag, "ms": round(ms, 4),
                      "TBps": round((F * d // 2 + F * d * 2) / ms / 1e9, 3)}), flush=True)
    assert torch.equal(outT, out.t()), "transposed dequant != rows dequant transposed"


if __name__ == "__main__":
    main()
