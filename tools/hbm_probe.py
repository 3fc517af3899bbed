#!/usr/bin/env python3
"""Workload for the per-kernel HBM table (tools/pmc_run.sh hbm ... -- python3 tools/hbm_probe.py):
a calibration kernel of known traffic, then the 1-layer Llama-3-8B LoRA step (the per-layer kernels of
the headline step at its real shapes: B 4 x S 4096).

Calibration: ``torch.mul(a, 2.0, out=b)`` on 1 GiB bf16 tensors (kernel `vectorized_elementwise_kernel<8, AUnaryFunctor<..MulFunctor..>>`) (1 GiB read, 1 GiB written, streamed
once) -- its FETCH_SIZE / WRITE_SIZE counters give the bytes-per-count scale that tools/pmc_md.py
--hbm applies to every other kernel (gfx950's TCC counters tally requests, not bytes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = 1 << 29  # 2^29 bf16 = 1 GiB
    a = torch.rand(n, device="cuda").to(torch.bfloat16)
    b = torch.empty_like(a)
    for _ in range(3):
        torch.mul(a, 2.0, out=b)
    torch.cuda.synchronize()
    del a, b
    torch.cuda.empty_cache()
    from finetune_controller_amd.train.trainer import TrainConfig, Trainer

    tr = Trainer(TrainConfig(model="llama3-8b-1l", method="lora", batch_size=4, seq_len=4096, synthetic=True,
                             max_steps=3, save_model=False, resume=False, device="cuda"))
    for _ in range(2):
        tr.train_step(1e-4)
    torch.cuda.synchronize()
    tr.close()
    print("[hbm_probe] done")


if __name__ == "__main__":
    main()
