#!/usr/bin/env python3
"""Learnable synthetic corpus for convergence checks (no datasets offline): windows made of one random
chunk repeated (an induction / copy task), tokens from a vocabulary subset.  Writes a 1-D int32 .npy.

    python tools/make_structured_tokens.py OUT.npy [--tokens 4000000] [--chunk 128] [--vocab 2000] [--mode copy|pairs]

Every window's first chunk is unpredictable (loss ~ ln(vocab)); every later token is a copy of the
token one chunk back -- a model that learns induction drives the loss toward
ln(vocab) / repeats_per_window."""
import argparse

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--tokens", type=int, default=4_000_000)
    ap.add_argument("--chunk", type=int, default=128)
    ap.add_argument("--window", type=int, default=2048)
    ap.add_argument("--vocab", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--mode", default="copy", choices=["copy", "pairs"],
                    help="pairs: every token appears twice in a row (a a b b ...): the second of each pair is the "
                         "previous position's token -- learnable only through attention; ideal loss ln(vocab)/2")
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    if a.mode == "pairs":
        half = rng.integers(3, a.vocab, size=(a.tokens + 1) // 2, dtype=np.int32)
        data = np.repeat(half, 2)[: a.tokens]
        np.save(a.out, data.astype(np.int32), allow_pickle=False)
        print(f"{a.out}: {data.size} tokens, repeated pairs over {a.vocab} ids")
        return
    nwin = -(-a.tokens // a.window)
    chunks = rng.integers(3, a.vocab, size=(nwin, a.chunk), dtype=np.int32)
    reps = a.window // a.chunk
    data = np.tile(chunks, (1, reps)).reshape(-1)[: a.tokens]
    np.save(a.out, data.astype(np.int32), allow_pickle=False)
    print(f"{a.out}: {data.size} tokens, {nwin} windows of {reps} x {a.chunk}-token chunks")


if __name__ == "__main__":
    main()
