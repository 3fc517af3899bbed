#!/usr/bin/env python3
"""Where the projection GEMM's K loop waits: runs the FTC_GEMM_STAMP build (tools/gemm_lab/build_stamp.sh)
through ctypes on the headline step's shapes and prints, per shape, the mean share of the loop's wave
cycles spent in each wait segment (first 8 workgroups x 4 waves):

  lgkm1 / bar1  -- Y.A fragment reads retired / the A-region release barrier
  lgkm2 / bar2  -- Y.B fragment reads retired / the B-region release barrier
  vm / bar3     -- the next stage's DMA landed (counted vmcnt) / the publish barrier

    python tools/gemm_lab/stamps.py [--shapes qkv_fwd,gu_fwd] [--configs "0,-8,32,0;100000,-8,32,0"]

The stamps (s_memtime + lgkmcnt(0)) add their own cost (guide "In-kernel stamps": shares, not lengths);
the same binary's time per call is printed beside them."""
import argparse
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tools.bench_gemm_nt import SHAPES, T, timeit  # noqa: E402

NAMES = ["lgkm1", "bar1", "lgkm2", "bar2", "vm", "bar3"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="qkv_fwd,gu_fwd,down_fwd")
    ap.add_argument("--configs", default="0,-8,32,0;100000,-8,32,0")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(HERE, "libgemm_stamp.so"))
    lib.ftc_gemm_nt.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p,
                                ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
    lib.ftc_gemm_nt_config.argtypes = [ctypes.c_int] * 5
    lib.ftc_gemm_nt_stamps.argtypes = [ctypes.c_void_p]
    torch.manual_seed(0)
    for name in a.shapes.split(","):
        k, n = SHAPES[name]
        x = torch.empty(T, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        w = torch.empty(n, k, device="cuda", dtype=torch.bfloat16).uniform_(-1, 1)
        y = torch.empty(T, n, device="cuda", dtype=torch.bfloat16)
        ref = torch.mm(x, w.t())
        for cfg in a.configs.split(";"):
            lib.ftc_gemm_nt_config(*([int(v) for v in cfg.split(",")] + [0, 0])[:5])
            st = torch.cuda.current_stream().cuda_stream

            def run():
                rc = lib.ftc_gemm_nt(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), y.data_ptr(), y.stride(0),
                                     0, T, n, k, 1.0, 0.0, st)
                assert rc == 0, rc

            run()
            torch.cuda.synchronize()
            assert torch.equal(y, ref), name
            ms = timeit(run, a.iters)
            buf = (ctypes.c_ulonglong * (8 * 4 * 8))()
            assert lib.ftc_gemm_nt_stamps(buf) == 0
            rows = [[buf[(b * 4 + wv) * 8 + i] for i in range(8)] for b in range(8) for wv in range(4)]
            loop = sum(r[6] for r in rows)
            share = {nm: round(sum(r[i] for r in rows) / loop, 4) for i, nm in enumerate(NAMES)}
            iters = sum(r[7] for r in rows) / len(rows)
            print(json.dumps({"gemm": name, "config": cfg, "ms": round(ms, 4), "tf": round(2 * T * n * k / ms / 1e9),
                              "iters_per_wave": iters, "cycles_per_iter": round(loop / len(rows) / max(1, iters)),
                              "wait_share": share, "wait_total": round(sum(share.values()), 4)}), flush=True)
        del x, w, y, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
