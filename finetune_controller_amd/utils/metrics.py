"""Training metrics in the controller's format.

The monitor pulls the newest object whose key contains ``metrics`` and ends in ``.csv`` from the
job's artifact prefix and stores its rows (NaN -> 0) in Mongo
(``/root/reference/app/utils/S3Handler.py:237-292``, ``/root/reference/app/core/monitor.py:34-95``);
the UI links the exact basename ``metrics.csv`` (``/root/reference/app/main.py:700``).  The worker
therefore appends to ``<checkpoint_path>/metrics.csv`` and flushes every row, so the 60 s sidecar
sync always ships a consistent file.
"""
from __future__ import annotations

import csv
import os

COLUMNS = ["epoch", "step", "loss", "lr", "tokens_per_sec", "step_time_ms", "grad_norm", "world_size", "mem_gb",
           "tflops_per_gpu", "fwd_ms", "bwd_ms", "comm_ms", "optim_ms", "eval_loss"]


class MetricsCSV:
    def __init__(self, path: str, enabled: bool = True, resume: bool = False, resume_step: int | None = None):
        """``resume_step``: the step the run restarts after.  Rows past it were logged by the attempt that
        died after its last checkpoint; those steps run again, so they are dropped first (one row per
        step in the UI's curves, not two)."""
        self.path, self.enabled = path, enabled
        if not enabled:
            return
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        exists = os.path.exists(path) and os.path.getsize(path) > 0
        if resume and exists and resume_step is not None:
            _truncate_after(path, resume_step)
        self.f = open(path, "a" if (resume and exists) else "w", newline="")
        self.w = csv.DictWriter(self.f, fieldnames=COLUMNS, extrasaction="ignore")
        if not (resume and exists):
            self.w.writeheader()
            self.f.flush()

    def write(self, row: dict):
        if not self.enabled:
            return
        self.w.writerow({k: row.get(k, "") for k in COLUMNS})
        self.f.flush()

    def close(self):
        if self.enabled:
            self.f.close()


def _truncate_after(path: str, step: int) -> None:
    with open(path, newline="") as f:
        rows = list(csv.reader(f))
    if not rows or "step" not in rows[0]:
        return
    si = rows[0].index("step")
    keep = [rows[0]]
    for r in rows[1:]:
        try:
            if int(float(r[si])) > step:
                continue
        except (IndexError, ValueError):
            continue  # a torn last line from the crash
        keep.append(r)
    tmp = path + ".tmp"
    with open(tmp, "w", newline="") as f:
        csv.writer(f).writerows(keep)
    os.replace(tmp, path)


def read_metrics_csv(path: str) -> list[dict]:
    """Records with NaN/empty -> 0 (the monitor's ingestion semantics)."""
    out = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rec = {}
            for k, v in r.items():
                try:
                    x = float(v)
                    if x != x:
                        x = 0.0
                    rec[k] = int(x) if x.is_integer() and k in ("epoch", "step", "world_size") else x
                except (TypeError, ValueError):
                    rec[k] = 0 if v in ("", None, "nan", "NaN") else v
            out.append(rec)
    return out
