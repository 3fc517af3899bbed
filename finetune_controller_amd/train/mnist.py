"""The reference's example job, runnable on this framework's worker image.

The reference registers exactly one model, ``MNIST`` (``/root/reference/app/models/examples/mnist.py:13-99``),
whose container is an external image running ``python mnist_training_script.py`` with the flags
``--batch-size --test-batch-size --epochs --lr --gamma --seed --log-interval [--no-cuda] [--save-model]``
(``mnist.py:77-99``) plus the mount contract ``--dataset_path`` / ``--checkpoint_path``.  This module
accepts exactly that command line, so the same job spec (``MNIST-MI355X`` in
``controlplane/spec/models/builtin.py``) runs here: a small CNN classifier (two 3x3 convolutions,
max-pool, two linear layers; Adadelta + per-epoch StepLR), one process per GPU under ``torchrun``
with gradients averaged by ``DistributedDataParallel`` (RCCL on MI355X, gloo on CPU).

Data: IDX files (``train-images-idx3-ubyte[.gz]`` ...) or ``mnist.npz`` (``x_train`` ...) under
``--dataset_path``; without them (no network here) a seeded synthetic digit set of the same shape --
ten class templates, random shifts and noise -- that the network learns in one epoch.

Outputs in ``--checkpoint_path``: ``metrics.csv`` (epoch, step, loss, lr, test_loss, accuracy, ...),
``Train Epoch: ...`` log lines (the UI stream starts at the first line containing ``Epoch``), and
``mnist_cnn.pt`` (a ``state_dict``) with ``--save-model``.
"""
from __future__ import annotations

import argparse
import csv
import gzip
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..parallel import dist as pdist

MEAN, STD = 0.1307, 0.3081


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.drop1 = nn.Dropout(0.25)
        self.drop2 = nn.Dropout(0.5)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, 10)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = self.drop1(torch.flatten(x, 1))
        x = self.drop2(F.relu(self.fc1(x)))
        return F.log_softmax(self.fc2(x), dim=1)


# ------------------------------------------------------------------ data
def _read_idx(path: str) -> np.ndarray:
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rb") as f:
        raw = f.read()
    magic = int.from_bytes(raw[0:4], "big")
    ndim = magic & 0xFF
    if (magic >> 8) != 0x08:  # unsigned byte payload
        raise ValueError(f"{path}: unsupported IDX type 0x{magic:08x}")
    dims = [int.from_bytes(raw[4 + 4 * i: 8 + 4 * i], "big") for i in range(ndim)]
    return np.frombuffer(raw, dtype=np.uint8, offset=4 + 4 * ndim).reshape(dims)


def _find(root: str, stem: str) -> str | None:
    for dp, _, files in os.walk(root):
        for f in files:
            if f.startswith(stem) and (f.endswith("ubyte") or f.endswith("ubyte.gz")):
                return os.path.join(dp, f)
    return None


def synthetic_mnist(n: int, seed: int) -> tuple[np.ndarray, np.ndarray]:
    """[n, 28, 28] uint8 images of 10 fixed class templates (blurred random strokes) shifted by up to
    3 pixels with additive noise, and their labels."""
    g = np.random.default_rng(1234)  # the templates are the same for every split
    tmpl = np.zeros((10, 28, 28), np.float32)
    for c in range(10):
        for _ in range(4):  # four random line segments per class
            (r0, c0), (r1, c1) = g.integers(6, 22, size=(2, 2))
            for t in np.linspace(0.0, 1.0, 24):
                r, cc = int(round(r0 + t * (r1 - r0))), int(round(c0 + t * (c1 - c0)))
                tmpl[c, r - 1:r + 2, cc - 1:cc + 2] = 1.0
    r = np.random.default_rng(seed)
    y = r.integers(0, 10, size=n)
    dx, dy = r.integers(-3, 4, size=n), r.integers(-3, 4, size=n)
    x = np.empty((n, 28, 28), np.float32)
    for i in range(n):
        x[i] = np.roll(np.roll(tmpl[y[i]], dy[i], 0), dx[i], 1)
    x = np.clip(x * 0.8 + r.normal(0.0, 0.15, size=x.shape), 0.0, 1.0)
    return (x * 255).astype(np.uint8), y.astype(np.int64)


def load_mnist(path: str, train_size: int, test_size: int, seed: int):
    """(x_train, y_train, x_test, y_test, source) with uint8 images."""
    if path and os.path.isdir(path):
        files = {k: _find(path, k) for k in ("train-images", "train-labels", "t10k-images", "t10k-labels")}
        if all(files.values()):
            return (_read_idx(files["train-images"]), _read_idx(files["train-labels"]).astype(np.int64),
                    _read_idx(files["t10k-images"]), _read_idx(files["t10k-labels"]).astype(np.int64), "idx")
        for dp, _, fs in os.walk(path):
            if "mnist.npz" in fs:
                with np.load(os.path.join(dp, "mnist.npz"), allow_pickle=False) as z:
                    return (z["x_train"], z["y_train"].astype(np.int64), z["x_test"], z["y_test"].astype(np.int64),
                            "npz")
    xtr, ytr = synthetic_mnist(train_size, seed)
    xte, yte = synthetic_mnist(test_size, seed + 1)
    return xtr, ytr, xte, yte, "synthetic"


def _to_tensor(x: np.ndarray, device) -> torch.Tensor:
    t = torch.from_numpy(np.ascontiguousarray(x)).to(device).float().div_(255.0)
    return t.sub_(MEAN).div_(STD).unsqueeze(1)


# ------------------------------------------------------------------ loop
def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="ftc-mnist", description="MNIST example job (reference example contract)")
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--test-batch-size", type=int, default=1000)
    ap.add_argument("--epochs", type=int, default=14)
    ap.add_argument("--lr", type=float, default=1.0)
    ap.add_argument("--gamma", type=float, default=0.7)
    ap.add_argument("--no-cuda", action="store_true")
    ap.add_argument("--no-mps", action="store_true")  # accepted for command-line compatibility
    ap.add_argument("--dry-run", action="store_true", help="one batch per epoch")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--log-interval", type=int, default=10)
    ap.add_argument("--save-model", action="store_true")
    ap.add_argument("--train-size", type=int, default=60000, help="synthetic training images (no dataset)")
    ap.add_argument("--test-size", type=int, default=10000, help="synthetic test images (no dataset)")
    ap.add_argument("--dataset_path", "--dataset-path", dest="dataset_path", default="/data/dataset")
    ap.add_argument("--checkpoint_path", "--checkpoint-path", dest="checkpoint_path", default="/data/artifacts")
    return ap


def run(a) -> dict:
    info = pdist.init_distributed("cpu" if a.no_cuda else "auto")
    dev = info.device
    torch.manual_seed(a.seed)
    xtr, ytr, xte, yte, src = load_mnist(a.dataset_path, a.train_size, a.test_size, a.seed)
    # each rank trains on its strided shard; the test set is scored whole on every rank
    # (equal shard sizes: every rank runs the same number of DDP steps)
    keep = len(xtr) // info.world_size * info.world_size
    xtr, ytr = xtr[info.rank:keep:info.world_size], ytr[info.rank:keep:info.world_size]
    Xtr, Ytr = _to_tensor(xtr, dev), torch.from_numpy(ytr).to(dev)
    Xte, Yte = _to_tensor(xte, dev), torch.from_numpy(yte).to(dev)
    model = Net().to(dev)
    net = model
    if info.distributed:  # DDP broadcasts rank 0's weights and averages gradients in buckets
        net = nn.parallel.DistributedDataParallel(model, device_ids=[dev.index] if dev.type == "cuda" else None)
    opt = torch.optim.Adadelta(net.parameters(), lr=a.lr)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=a.gamma)
    os.makedirs(a.checkpoint_path, exist_ok=True)
    cols = ["epoch", "step", "loss", "lr", "test_loss", "accuracy", "samples_per_sec", "world_size"]
    fcsv = open(os.path.join(a.checkpoint_path, "metrics.csv"), "w", newline="") if info.is_main else None
    wcsv = csv.DictWriter(fcsv, fieldnames=cols) if fcsv else None
    if wcsv:
        wcsv.writeheader()
        print(f"mnist: data={src} train={len(Xtr) * info.world_size} test={len(Xte)} device={dev} "
              f"world={info.world_size}", flush=True)
    n = len(Xtr)
    nb = (n + a.batch_size - 1) // a.batch_size
    step, last = 0, {}
    g = torch.Generator().manual_seed(a.seed)
    for epoch in range(1, a.epochs + 1):
        net.train()
        perm = torch.randperm(n, generator=g).to(dev)
        t0 = time.perf_counter()
        for bi in range(nb):
            idx = perm[bi * a.batch_size:(bi + 1) * a.batch_size]
            opt.zero_grad(set_to_none=True)
            loss = F.nll_loss(net(Xtr[idx]), Ytr[idx])
            loss.backward()
            opt.step()
            step += 1
            if bi % a.log_interval == 0 or a.dry_run:
                lv = float(loss.detach())
                seen = bi * a.batch_size * info.world_size
                if wcsv:
                    print(f"Train Epoch: {epoch} [{seen}/{n * info.world_size} ({100.0 * bi / nb:.0f}%)]\t"
                          f"Loss: {lv:.6f}", flush=True)
                    wcsv.writerow({"epoch": epoch, "step": step, "loss": round(lv, 6),
                                   "lr": opt.param_groups[0]["lr"], "world_size": info.world_size,
                                   "samples_per_sec": round((bi + 1) * a.batch_size * info.world_size /
                                                            max(time.perf_counter() - t0, 1e-9), 1)})
                    fcsv.flush()
            if a.dry_run:
                break
        # test
        net.eval()
        tot, correct = 0.0, 0
        with torch.no_grad():
            for i in range(0, len(Xte), a.test_batch_size):
                out = model(Xte[i:i + a.test_batch_size])
                tot += float(F.nll_loss(out, Yte[i:i + a.test_batch_size], reduction="sum"))
                correct += int((out.argmax(1) == Yte[i:i + a.test_batch_size]).sum())
        test_loss, acc = tot / len(Xte), 100.0 * correct / len(Xte)
        last = {"epoch": epoch, "step": step, "test_loss": round(test_loss, 6), "accuracy": round(acc, 3),
                "lr": opt.param_groups[0]["lr"], "world_size": info.world_size}
        if wcsv:
            print(f"\nTest set (Epoch {epoch}): Average loss: {test_loss:.4f}, Accuracy: {correct}/{len(Xte)} "
                  f"({acc:.0f}%)\n", flush=True)
            wcsv.writerow(last)
            fcsv.flush()
        sched.step()
    if a.save_model and info.is_main:
        torch.save(model.state_dict(), os.path.join(a.checkpoint_path, "mnist_cnn.pt"))
    if fcsv:
        fcsv.close()
    pdist.barrier(info)
    pdist.destroy(info)
    return last


def main(argv=None) -> int:
    last = run(build_parser().parse_args(argv))
    print(f"Training complete: {last}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
