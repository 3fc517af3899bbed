"""Token data for the worker: synthetic streams (benchmarks) and the dataset the controller's
init container drops into ``/data/dataset`` (``/root/reference/app/jobs/kubeflow/PyTorchJobDeployer.py:70-91``).

Dataset formats accepted in ``--dataset_path`` (a file, or a directory holding one):

* ``*.bin`` / ``*.tokens``  -- raw little-endian uint16 (vocab <= 65536) or uint32 token ids
  (``.u32.bin``), memory-mapped and packed by the native loader (``csrc/runtime/token_loader.cpp``);
* ``*.npy``                 -- 1-D integer token array (``allow_pickle=False``);
* ``*.jsonl`` / ``*.json``  -- records with a ``text`` field (or ``prompt``/``completion``);
* ``*.txt`` / ``*.csv``     -- text, one sample per line (CSV: first text-like column).

Text is tokenised with a ``tokenizer.json`` found next to the data (HF ``tokenizers``) or, failing
that, a byte-level fallback (ids = bytes + 3, so the vocab must be >= 259).  Samples are packed into
fixed ``[batch, seq_len]`` blocks with next-token labels.
"""
from __future__ import annotations

import csv
import glob
import json
import os
from pathlib import Path

import numpy as np
import torch


class SyntheticTokens:
    """Uniform random token ids of the configured shape (the benchmark contract's synthetic data).

    Every step draws a FRESH batch on the device from a generator re-seeded with (seed, step): no
    host->device copy in the timed loop, nothing the model could memorise (a small cycled pool lets
    the loss fall below ln(vocab)), and a resumed run sees the same stream.  Packed-document mode
    (``doc_len``) keeps a 4-batch pool whose label masks are precomputed."""

    def __init__(self, vocab: int, batch: int, seq_len: int, device, seed: int = 0, doc_len: int = 0,
                 eos_id: int = 2):
        self.vocab, self.batch, self.seq_len, self.device = vocab, batch, seq_len, device
        self.seed = int(seed)
        self.gen = torch.Generator(device="cpu").manual_seed(seed)
        self.last_n_valid, self.labels, self.pool = None, None, None
        if doc_len:  # packed documents of doc_len tokens: EOS at the end of each (its label ignored)
            pool = [torch.randint(0, vocab, (batch, seq_len + 1), generator=self.gen) for _ in range(4)]
            for t in pool:
                t[t == eos_id] = (eos_id + 1) % vocab
                t[:, doc_len - 1::doc_len] = eos_id
            self.labels = [t[:, 1:].masked_fill(t[:, :-1] == eos_id, -100).to(device) for t in pool]
            self.last_n_valid = int((self.labels[0] != -100).sum().item())
            self.pool = [t.to(device) for t in pool]
        else:
            self._dgen = torch.Generator(device=device)
        self.i = 0

    def __iter__(self):
        return self

    def __next__(self):
        if self.pool is not None:
            t = self.pool[self.i % len(self.pool)]
            y = self.labels[self.i % len(self.pool)]
        else:
            self._dgen.manual_seed(self.seed * 1_000_003 + self.i)
            t = torch.randint(0, self.vocab, (self.batch, self.seq_len + 1), device=self.device, generator=self._dgen)
            y = t[:, 1:]
        self.i += 1
        return t[:, :-1], y

    def state(self):
        return {"i": self.i}

    def load_state(self, st):
        self.i = int(st.get("i", 0))


def _find_data_file(path: str) -> str | None:
    if not path or not os.path.exists(path):
        return None
    if os.path.isfile(path):
        return path
    cands = []
    for pat in ("*.bin", "*.tokens", "*.npy", "*.jsonl", "*.json", "*.txt", "*.csv"):
        cands += sorted(glob.glob(os.path.join(path, "**", pat), recursive=True))
    cands = [c for c in cands if not os.path.basename(c).startswith("tokenizer")]
    return cands[0] if cands else None


def _field(v) -> str:
    return "" if v is None else str(v)


def _records(path: str):
    """(prompt, completion) per record: ``prompt`` is "" for plain text (loss on every token)."""
    ext = Path(path).suffix.lower()
    if ext in (".jsonl", ".json"):
        with open(path, encoding="utf-8-sig") as f:  # -sig: a UTF-8 byte-order mark is not part of the data
            head = f.read(64).lstrip()[:1]
            f.seek(0)
            rows = json.load(f) if (ext == ".json" and head == "[") else (json.loads(l) for l in f if l.strip())
            for n, r in enumerate(rows):
                if isinstance(r, str):
                    yield "", r
                elif not isinstance(r, dict):
                    raise ValueError(f"{path}: record {n} is a {type(r).__name__}; expected an object or a string")
                elif "text" in r:
                    yield "", _field(r["text"])
                else:
                    yield _field(r.get("prompt")), _field(r.get("completion", r.get("response")))
    elif ext == ".csv":
        with open(path, encoding="utf-8-sig", newline="") as f:
            rd = csv.reader(f)
            header = next(rd, None)
            col = 0
            if header:
                for i, h in enumerate(header):
                    if h.lower() in ("text", "smiles", "sequence", "prompt", "content"):
                        col = i
                        break
            for row in rd:
                if len(row) > col:  # blank and short (ragged) rows carry no text
                    yield "", row[col]
    else:
        with open(path, encoding="utf-8", errors="replace") as f:
            for line in f:
                if line.strip():
                    yield "", line.rstrip("\n")


class Tokenizer:
    def __init__(self, data_path: str | None, vocab: int):
        self.vocab = vocab
        self.tk = None
        self.eos = 2
        cand = None
        if data_path:
            d = data_path if os.path.isdir(data_path) else os.path.dirname(data_path)
            p = os.path.join(d, "tokenizer.json")
            cand = p if os.path.exists(p) else None
        if cand:
            from tokenizers import Tokenizer as HFTok

            self.tk = HFTok.from_file(cand)
            for name in ("<|end_of_text|>", "</s>", "<|endoftext|>", "<eos>", "<|eot_id|>"):
                i = self.tk.token_to_id(name)
                if i is not None:
                    self.eos = int(i)
                    break
        elif vocab < 259:
            raise ValueError("byte-level fallback tokenizer needs vocab >= 259")

    def encode(self, text: str) -> list[int]:
        if self.tk is not None:
            return self.tk.encode(text).ids
        return [b + 3 for b in text.encode("utf-8")]

    def encode_batch(self, texts: list[str]) -> list[list[int]]:
        """``encode`` of every text; the HF tokenizer encodes the batch on its own thread pool."""
        if self.tk is not None:
            return [e.ids for e in self.tk.encode_batch(texts)]
        return [self.encode(t) for t in texts]


def check_token_ids(w: np.ndarray, vocab: int) -> np.ndarray:
    """A host batch of ids must lie in [0, vocab): an out-of-range id would make the embedding gather
    read outside the table -- a GPU memory fault, not an exception (the native loader checks the same
    per batch)."""
    if w.size and (int(w.max()) >= vocab or int(w.min()) < 0):
        raise ValueError(f"dataset token ids must lie in [0, {vocab}) for this model; found "
                         f"[{int(w.min())}, {int(w.max())}] (wrong tokenizer / vocabulary?)")
    return w


def load_token_array(path: str, vocab: int) -> np.ndarray:
    """Return a 1-D int array of token ids for a dataset path (memory-mapped when binary)."""
    return load_tokens_and_mask(path, vocab)[0]


def load_tokens_and_mask(path: str, vocab: int, completion_only: bool = False):
    """(ids, loss_mask): ``loss_mask`` (uint8, same length, or None) is 0 on prompt tokens of
    prompt/completion records when ``completion_only`` -- their next-token labels are not trained on."""
    f = _find_data_file(path)
    if f is None:
        raise FileNotFoundError(f"no dataset file under {path!r}")
    ext = Path(f).suffix.lower()
    if ext in (".bin", ".tokens"):
        dt = np.uint32 if f.endswith(".u32.bin") or vocab > 65536 else np.uint16
        return np.memmap(f, dtype=dt, mode="r"), None
    if ext == ".npy":
        return np.load(f, mmap_mode="r", allow_pickle=False), None
    tok = Tokenizer(path, vocab)
    # records are encoded TEXT_BATCH at a time into int32 / uint8 numpy chunks: 5 bytes per token resident,
    # ~10 at the peak (measured on a 20M-token JSONL: 10 vs 25 with whole-dataset Python int lists, more
    # than 25 once tokenizer ids exceed 256 and stop being shared small-int objects)
    ids_chunks: list[np.ndarray] = []
    mask_chunks: list[np.ndarray] = []
    batch: list[tuple[str, str]] = []

    def flush():
        enc_p = tok.encode_batch([p for p, _ in batch if p])
        enc_c = tok.encode_batch([c for _, c in batch])
        ip = iter(enc_p)
        ids: list[int] = []
        mask: list[int] = []
        for (prompt, _), c in zip(batch, enc_c):
            p = next(ip) if prompt else []
            ids += p
            ids += c
            ids.append(tok.eos)
            mask += [0] * len(p)
            mask += [1] * (len(c) + 1)
        ids_chunks.append(np.asarray(ids, dtype=np.int32))
        mask_chunks.append(np.asarray(mask, dtype=np.uint8))
        batch.clear()

    for rec in _records(f):
        batch.append(rec)
        if len(batch) >= TEXT_BATCH:
            flush()
    if batch:
        flush()
    arr = np.concatenate(ids_chunks) if ids_chunks else np.zeros(0, dtype=np.int32)
    if arr.size and (int(arr.max()) >= vocab or tok.eos >= vocab):
        # a tokenizer.json of a larger vocabulary than the model's: wrapping the ids would train on
        # scrambled tokens without a visible error
        raise ValueError(f"tokenizer ids reach {max(int(arr.max()), tok.eos)} but the model's vocabulary "
                         f"has {vocab} entries (tokenizer.json of another model?)")
    del ids_chunks
    m = np.concatenate(mask_chunks) if completion_only and mask_chunks else None
    return arr, (m if m is not None and not m.all() else None)


TEXT_BATCH = 1024  # records per tokenizer batch in load_tokens_and_mask


class PackedTokenDataset:
    """Fixed [batch, seq_len+1] windows over a token array, sharded by rank, epoch-shuffled.

    Uses the native loader (C++ thread pool, prefetching pinned batches) when ``_rt.so`` is built,
    otherwise numpy indexing.
    """

    def __init__(self, path: str, vocab: int, batch: int, seq_len: int, device, rank: int = 0, world: int = 1,
                 seed: int = 0, holdout: float = 0, eos_id: int | None = None, completion_only: bool = False):
        self.tokens, self.loss_mask = load_tokens_and_mask(path, vocab, completion_only)
        self.vocab, self.batch, self.seq_len, self.device = vocab, batch, seq_len, device
        self.rank, self.world, self.seed = rank, world, seed
        n_windows = (len(self.tokens) - 1) // seq_len
        if n_windows < 1:
            raise ValueError(f"dataset has {len(self.tokens)} tokens; need > seq_len={seq_len}")
        self.n_windows = n_windows
        # the last windows are an evaluation split (EvalWindows), never trained on: `holdout` is a share
        # of the windows (< 1) or a count, at least one micro-batch per rank
        want = 0
        if holdout > 0:
            want = max(int(holdout) if holdout >= 1 else int(round(n_windows * holdout)), batch * world)
        self.holdout = max(0, min(want, n_windows - 1))
        self.n_use = n_windows - self.holdout
        # label masking (host side, so the loss normaliser ``last_n_valid`` needs no device sync):
        # packed documents ignore the label of every EOS input (it would predict across a document
        # boundary), completion-only training the labels of prompt tokens
        self.eos_id, self.last_n_valid = eos_id, None
        self.steps_per_epoch = max(1, self.n_use // (batch * world))
        self.epoch = 0
        self.pos = 0
        self._native = None
        try:
            from ..utils.native import NativeTokenLoader

            dt = self.tokens.dtype
            if (isinstance(self.tokens, np.memmap) and self.loss_mask is None and dt.itemsize in (2, 4)
                    and (dt.kind == "u" or (dt.kind == "i" and dt.itemsize == 4))  # the loader reads unsigned:
                    # a negative int32 id wraps past any vocabulary and is rejected, a negative int16 one
                    # (-1 -> 65535) would pass a > 65535 vocabulary -- int16 files take the numpy path
                    and dt.byteorder in "=<|" and self.tokens.ndim == 1
                    and os.environ.get("FTC_NATIVE_LOADER", "1") != "0"):
                # offset: a .npy file's header precedes the tokens; vocab: ids are range-checked per batch
                self._native = NativeTokenLoader(self.tokens.filename, dt.itemsize, seq_len, batch, rank, world, seed,
                                                 n_use=self.n_use, offset=int(self.tokens.offset), vocab=vocab)
        except ImportError:  # _rt.so not built: numpy path
            self._native = None
        self._perm()

    def _perm(self):
        rng = np.random.default_rng(self.seed + self.epoch)
        self.order = rng.permutation(self.n_use)

    def __iter__(self):
        return self

    def __next__(self):
        if self._native is not None:
            arr = self._native.next_batch()  # [batch, seq_len+1] int64 (pinned)
            self.pos += 1
            if self.pos >= self.steps_per_epoch:
                self.pos, self.epoch = 0, self.epoch + 1
        else:
            if self.pos >= self.steps_per_epoch:
                self.pos, self.epoch = 0, self.epoch + 1
                self._perm()
            base = (self.pos * self.world + self.rank) * self.batch
            idx = [self.order[(base + i) % self.n_use] for i in range(self.batch)]
            arr = self._windows(idx)
            self.pos += 1
        labels = self._labels(arr, idx if self._native is None else None)
        if labels is not None:
            cpu = torch.device(self.device).type == "cpu"
            x = arr[:, :-1].clone() if cpu else arr[:, :-1].to(self.device, non_blocking=True)
            if self._native is not None and not cpu:
                self._native.copied()
            return x, labels.to(self.device, non_blocking=True)
        if self._native is not None:
            if torch.device(self.device).type == "cpu":
                t = arr.clone()  # the ring buffer is refilled after the next call
            else:
                t = arr.to(self.device, non_blocking=True)
                self._native.copied()
        else:
            t = arr.to(self.device, non_blocking=True)
        return t[:, :-1], t[:, 1:]

    def _windows(self, idx) -> torch.Tensor:
        S = self.seq_len
        w = np.stack([np.asarray(self.tokens[j * S: j * S + S + 1], dtype=np.int64) for j in idx])
        return torch.from_numpy(check_token_ids(w, self.vocab))

    def _labels(self, arr: torch.Tensor, idx) -> torch.Tensor | None:
        """Masked labels of a [batch, S+1] host window batch (None: no masking configured)."""
        if self.eos_id is None and self.loss_mask is None:
            return None
        y = arr[:, 1:].clone()
        if self.loss_mask is not None:
            S = self.seq_len
            m = torch.from_numpy(np.stack([self.loss_mask[j * S + 1: j * S + S + 1] for j in idx]))
            y[m == 0] = -100
        if self.eos_id is not None:
            y[arr[:, :-1] == self.eos_id] = -100
        self.last_n_valid = int((y != -100).sum())
        return y

    def state(self):
        return {"epoch": self.epoch, "pos": self.pos}

    def load_state(self, st):
        self.epoch, self.pos = int(st.get("epoch", 0)), int(st.get("pos", 0))
        self._perm()
        if self._native is not None:
            self._native.seek(self.epoch, self.pos)


class EvalWindows:
    """The held-out tail windows of a PackedTokenDataset as fixed evaluation batches: batch i of rank r
    takes windows ``n_use + ((i * world + r) * batch + j) % holdout`` -- the same every evaluation, so
    successive eval losses are comparable."""

    def __init__(self, ds: "PackedTokenDataset", n_batches: int):
        self.ds, self.n_batches = ds, max(1, int(n_batches))

    def batches(self):
        ds = self.ds
        if ds.holdout <= 0:
            return
        S = ds.seq_len
        for i in range(self.n_batches):
            base = (i * ds.world + ds.rank) * ds.batch
            idx = [ds.n_use + (base + j) % ds.holdout for j in range(ds.batch)]
            arr = ds._windows(idx)
            y = ds._labels(arr, idx)
            t = arr.to(ds.device, non_blocking=True)
            yield t[:, :-1], (t[:, 1:] if y is None else y.to(ds.device, non_blocking=True))
