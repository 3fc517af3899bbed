"""Kernel backend selection for the worker runtime.

Every hot op in :mod:`finetune_controller_amd.ops` has two implementations:

* the **HIP path** -- hand-written gfx950 kernels compiled into the in-tree
  extension ``finetune_controller_amd/_C*.so`` (sources under ``csrc/``);
* the **torch path** -- a plain PyTorch composition used on CPU (unit tests,
  the CPU-only FakeCluster e2e job) and as the numerics oracle.

Policy (deliberately strict so that a GPU run can never silently measure the
eager fallback):

* CPU tensors always take the torch path.
* GPU tensors take the HIP path.  If the extension is missing or fails to load
  on a GPU box we raise, unless ``FTC_KERNELS=torch`` is set explicitly -- the
  documented switch used to measure the "stock PyTorch-ROCm" baseline row of
  BASELINE.md.

The reference repository has no kernels at all; this module is
the seam the survey's K1..K11 kernels plug into.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch

_lock = threading.Lock()
_ext = None
_ext_error: BaseException | None = None


def kernel_mode() -> str:
    """``hip`` (default) or ``torch`` (forced stock-PyTorch path)."""
    mode = os.environ.get("FTC_KERNELS", "hip").strip().lower()
    if mode not in ("hip", "torch"):
        raise ValueError(f"FTC_KERNELS must be 'hip' or 'torch', got {mode!r}")
    return mode


def load_ext(required: bool = True):
    """Import the compiled HIP extension (``finetune_controller_amd._C``)."""
    global _ext, _ext_error
    if _ext is not None:
        return _ext
    with _lock:
        if _ext is None and _ext_error is None:
            try:
                _ext = importlib.import_module("finetune_controller_amd._C")
            except BaseException as e:  # ImportError, OSError (bad .so)
                _ext_error = e
    if _ext is None and required:
        raise RuntimeError(
            "finetune_controller_amd HIP extension is not available "
            f"({_ext_error!r}). Build it with `python -m finetune_controller_amd.tools.build` "
            "(or __graft_entry__.build()). Set FTC_KERNELS=torch to run the stock-PyTorch path on purpose."
        ) from _ext_error
    return _ext


def ext_available() -> bool:
    return load_ext(required=False) is not None


def use_hip(*tensors: torch.Tensor) -> bool:
    """True when the HIP kernels must handle these tensors."""
    t = next((x for x in tensors if isinstance(x, torch.Tensor)), None)
    if t is None or not t.is_cuda:
        return False
    if kernel_mode() == "torch":
        return False
    load_ext(required=True)  # fail loudly on a GPU box without the extension
    return True


def ext():
    return load_ext(required=True)


def stream_ptr(device: torch.device | None = None) -> int:
    """Raw hipStream_t of the current torch stream (kernels launch on it)."""
    return torch.cuda.current_stream(device).cuda_stream
