#!/usr/bin/env python3
"""The training script of walkthrough A (what the custom image runs): honours the controller <-> trainer
contract with numpy only.

* flags: the spec's training arguments plus ``--dataset_path`` / ``--checkpoint_path``;
* the dataset is one file the init container copied into ``--dataset_path`` (a directory);
* ``metrics.csv`` in ``--checkpoint_path`` (the monitor ingests it; the UI links it);
* log lines containing ``Epoch`` (the WebSocket log stream starts at the first one);
* artifacts matching the spec's ``store_asset_patterns`` (``model.json`` here);
* the controller appends ``&& touch done.txt`` itself -- exit 0 on success, non-zero on failure.
"""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--epochs", type=int, default=20)
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--l2", type=float, default=1e-4)
    ap.add_argument("--target-column", default="solubility")
    ap.add_argument("--dataset_path", required=True)
    ap.add_argument("--checkpoint_path", required=True)
    a = ap.parse_args(argv)
    files = sorted(glob.glob(os.path.join(a.dataset_path, "*.csv"))) if os.path.isdir(a.dataset_path) else [a.dataset_path]
    if not files:
        print(f"no CSV dataset under {a.dataset_path}", file=sys.stderr)
        return 2
    with open(files[0]) as f:
        rows = list(csv.DictReader(f))
    cols = [c for c in rows[0] if c != a.target_column]
    x = np.array([[float(r[c]) for c in cols] for r in rows])
    y = np.array([float(r[a.target_column]) for r in rows])
    mu, sd = x.mean(0), x.std(0) + 1e-8
    x = (x - mu) / sd
    w, b = np.zeros(x.shape[1]), float(y.mean())
    os.makedirs(a.checkpoint_path, exist_ok=True)
    with open(os.path.join(a.checkpoint_path, "metrics.csv"), "w", newline="") as f:
        out = csv.writer(f)
        out.writerow(["epoch", "loss", "lr"])
        for ep in range(a.epochs):
            err = x @ w + b - y
            loss = float((err ** 2).mean() + a.l2 * (w ** 2).sum())
            w -= a.lr * (2 * x.T @ err / len(y) + 2 * a.l2 * w)
            b -= a.lr * float(2 * err.mean())
            out.writerow([ep, f"{loss:.6f}", a.lr])
            f.flush()
            print(f"Epoch {ep}: loss={loss:.5f}", flush=True)
    with open(os.path.join(a.checkpoint_path, "model.json"), "w") as f:
        json.dump({"columns": cols, "mean": mu.tolist(), "std": sd.tolist(), "w": w.tolist(), "b": b}, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())
