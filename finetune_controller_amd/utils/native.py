"""Python side of the native token loader (``csrc/runtime/token_loader.cpp`` -> ``_rt.so``).

The C++ pool gathers the next batches of fixed windows from the memory-mapped token file into a
ring of pinned host buffers while the GPU trains; ``next_batch`` hands out the oldest ready buffer.
The window permutation is drawn here with numpy exactly like ``train.data.PackedTokenDataset``'s
fallback path, so both paths yield identical batches (tested in tests/test_worker.py).

A buffer is returned to the pool only after the device copy issued from it has completed (an event
recorded by :meth:`copied`), so the async H2D DMA never reads a buffer being refilled.
"""
from __future__ import annotations

import importlib

import numpy as np
import torch


def load_rt():
    return importlib.import_module("finetune_controller_amd._rt")


class NativeTokenLoader:
    def __init__(self, filename: str, itemsize: int, seq_len: int, batch: int, rank: int = 0, world: int = 1,
                 seed: int = 0, depth: int = 4, threads: int = 2, pin: bool | None = None, n_use: int | None = None,
                 offset: int = 0, vocab: int = 0):
        rt = load_rt()
        # offset: header bytes before the first token (.npy); vocab: ids >= vocab fail the batch on the host
        self.L = rt.TokenLoader(str(filename), int(itemsize), int(seq_len), int(batch), int(rank), int(world),
                                int(threads), int(offset), int(vocab))
        self.seq_len, self.batch, self.world, self.seed = seq_len, batch, world, seed
        self.n_windows = int(self.L.n_windows)
        # train on the first n_use windows only (the tail is a held-out evaluation split)
        self.n_use = min(self.n_windows, int(n_use)) if n_use else self.n_windows
        self.steps_per_epoch = max(1, self.n_use // (batch * world))
        if pin is None:
            pin = torch.cuda.is_available()
        self.bufs = [torch.empty(batch, seq_len + 1, dtype=torch.int64, pin_memory=pin) for _ in range(depth)]
        self.L.set_buffers([b.data_ptr() for b in self.bufs])
        self.events: list[torch.cuda.Event | None] = [None] * depth
        self.epoch, self.pos = 0, 0
        self._held: int | None = None
        self._start()

    def _order(self, epoch: int) -> np.ndarray:
        perm = np.random.default_rng(self.seed + epoch).permutation(self.n_use).astype(np.int64)
        if self.n_use == self.n_windows:
            return perm
        # batches only index the first n_use entries; the rest pads the array to the loader's length
        return np.concatenate([perm, np.arange(self.n_use, self.n_windows, dtype=np.int64)])

    def _start(self):
        self.L.start(self._order(self.epoch), self.pos, self.steps_per_epoch)

    def _release_held(self):
        if self._held is None:
            return
        ev = self.events[self._held]
        if ev is not None:
            ev.synchronize()
        self.L.release(self._held)
        self._held = None

    def next_batch(self) -> torch.Tensor:
        """[batch, seq_len + 1] int64 host tensor (pinned on GPU hosts), valid until the next call."""
        self._release_held()
        slot = self.L.acquire()
        if slot < 0:  # epoch done: new permutation
            self.epoch, self.pos = self.epoch + 1, 0
            self._start()
            slot = self.L.acquire()
        self.pos += 1
        self._held = slot
        self.events[slot] = None
        return self.bufs[slot]

    def copied(self):
        """Record that the device copy of the current batch has been queued on the current stream."""
        if self._held is not None and torch.cuda.is_available():
            ev = torch.cuda.Event()
            ev.record()
            self.events[self._held] = ev

    def seek(self, epoch: int, pos: int):
        self._release_held()
        self.L.stop()
        self.epoch, self.pos = int(epoch), int(pos)
        self._start()

    def close(self):
        self._release_held()
        self.L.stop()
