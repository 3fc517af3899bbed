#!/usr/bin/env python3
"""NF4 decode bandwidth at the Mistral-7B projection shapes: the row decode (forward operand) and the
transposed decode (TN backward operand) of csrc/kernels/nf4.hip, as used by ops/nf4.py per call.  Bytes =
0.5 (codes) + 2 (bf16 out) per parameter (+ the absmax bytes).  One JSON line per shape.

    python tools/bench_nf4_decode.py [--iters 50] [--shapes gate_up] [--ref]

--ref adds write-roof references on the same output views: ``fill`` (torch fill_ of the row view), ``copy``
(a bf16 [N, K] copied into the row view: 2 + 2 bytes per element) and ``rows_dense`` (the row decode into a
contiguous [N, K] buffer instead of the padded augmented operand).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from finetune_controller_amd.ops import nf4  # noqa: E402
from finetune_controller_amd.ops._backend import ext  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--ref", action="store_true")
    a = ap.parse_args()
    C = ext()
    torch.manual_seed(0)
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        qw = nf4.NF4Weight.quantize((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16))
        fwd = torch.empty(N + 64, K + 64, device="cuda", dtype=torch.bfloat16)
        bwdT = torch.empty(K, N + 64, device="cuda", dtype=torch.bfloat16)
        out = {}
        jobs = [("rows", fwd[:N, :K], False), ("t", bwdT[:, :N], True)]
        if a.ref:
            dense = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
            src = torch.randn(N, K, device="cuda").to(torch.bfloat16)
            jobs += [("rows_dense", dense, False), ("fill", fwd[:N, :K], "fill"), ("copy", fwd[:N, :K], "copy")]
        for tag, buf, tr in jobs:
            def run(buf=buf, tr=tr):
                if tr == "fill":
                    buf.fill_(1.0)
                elif tr == "copy":
                    buf.copy_(src)
                else:
                    C.nf4_dequantize_into(qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, buf, N, K, 64,
                                          qw.block2, tr)
            run()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                run()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / a.iters * 1000
            nbytes = {"fill": N * K * 2, "copy": N * K * 4}.get(tag, N * K * 2.5 + N * K / 64)
            out[tag] = {"us": round(us, 1), "TBps": round(nbytes / us / 1e6, 2)}
        ref = qw.dequantize()
        if a.ref:
            C.nf4_dequantize_into(qw.packed, qw.absmax_q, qw.absmax_scale, qw.absmax_offset, fwd[:N, :K], N, K, 64,
                                  qw.block2, False)
        ok = torch.equal(fwd[:N, :K], ref) and torch.equal(bwdT[:, :N], ref.t())
        if a.ref:
            ok = ok and torch.equal(dense, ref)
        print(json.dumps({"shape": name, "N": N, "K": K, **out, "exact": ok}), flush=True)


if __name__ == "__main__":
    main()
