#!/usr/bin/env python3
"""NF4 decode bandwidth at the Mistral-7B projection shapes: the row decode (forward operand) and the
transposed decode (TN backward operand) of csrc/kernels/nf4.hip, as used by ops/nf4.py per call.  Bytes =
0.5 (codes) + 2 (bf16 out) per parameter (+ the absmax bytes).  One JSON line per shape.

    python tools/bench_nf4_decode.py [--iters 50]
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
    a = ap.parse_args()
    C = ext()
    torch.manual_seed(0)
    for name, (N, K) in SHAPES.items():
        qw = nf4.NF4Weight.quantize((torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16))
        fwd = torch.empty(N + 64, K + 64, device="cuda", dtype=torch.bfloat16)
        bwdT = torch.empty(K, N + 64, device="cuda", dtype=torch.bfloat16)
        out = {}
        for tag, buf, tr in (("rows", fwd[:N, :K], False), ("t", bwdT[:, :N], True)):
            def run():
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
            nbytes = N * K * 2.5 + N * K / 64
            out[tag] = {"us": round(us, 1), "TBps": round(nbytes / us / 1e6, 2)}
        ref = qw.dequantize()
        ok = torch.equal(fwd[:N, :K], ref) and torch.equal(bwdT[:, :N], ref.t())
        print(json.dumps({"shape": name, "N": N, "K": K, **out, "exact": ok}), flush=True)


if __name__ == "__main__":
    main()
