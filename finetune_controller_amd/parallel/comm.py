"""Native RCCL engine front-end (N1/N2; C++ in ``csrc/comm/rccl_engine.cpp`` -> ``_comm.so``).

``NativeComm`` owns this process's RCCL communicator and a dedicated highest-priority HIP stream.
Collectives are ordered after the caller's queued work with an event and complete with an event the
caller's stream waits on *on the device* (``Work.wait()``), so gradient buckets all-reduce while the
rest of the backward pass keeps the CUs busy and nothing on the gradient path blocks the host.

Bootstrap: rank 0 draws the RCCL unique id, the id travels through torch.distributed (the c10d
store of the default group), every rank calls ``ncclCommInitRank``.  The torch process group stays
up for everything else (barriers, object broadcasts, the CPU/gloo path).

Used by ``parallel.ddp.GradBucketer(engine="native")`` and ``tools/comm_bench.py``.
"""
from __future__ import annotations

import importlib

import torch
import torch.distributed as dist


def load_comm():
    try:
        return importlib.import_module("finetune_controller_amd._comm")
    except ImportError as e:  # pragma: no cover - depends on the build
        raise RuntimeError("native RCCL engine not built: run `python -m finetune_controller_amd.tools.build`") from e


class Work:
    __slots__ = ("eng", "h")

    def __init__(self, eng, h: int):
        self.eng, self.h = eng, h

    def wait(self):
        """The current stream waits for the collective (device-side; returns immediately)."""
        self.eng.wait(self.h)

    def synchronize(self):
        self.eng.synchronize(self.h)

    def is_completed(self) -> bool:
        return self.eng.query(self.h)


class NativeComm:
    def __init__(self, group=None, device: torch.device | None = None):
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("NativeComm needs torch.distributed initialised (rendezvous + id exchange)")
        self._c = load_comm()
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        obj = [self._c.unique_id() if self.rank == 0 else None]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group, device=dev if dist.get_backend(group) == "nccl" else None)
        self.eng = self._c.Engine(obj[0], self.rank, self.world, dev.index)

    # ---- collectives (all asynchronous; .wait() orders the current stream after them)
    def all_reduce_async(self, t: torch.Tensor, op: str = "sum") -> Work:
        return Work(self.eng, self.eng.all_reduce(t, op))

    def broadcast_async(self, t: torch.Tensor, root: int = 0) -> Work:
        return Work(self.eng, self.eng.broadcast(t, root))

    def all_gather_async(self, out: torch.Tensor, inp: torch.Tensor) -> Work:
        return Work(self.eng, self.eng.all_gather(out, inp))

    def reduce_scatter_async(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum") -> Work:
        return Work(self.eng, self.eng.reduce_scatter(out, inp, op))

    def reset(self):
        """Recycle completion events (call once per step after every wait)."""
        self.eng.reset()

    def bench_all_reduce(self, t: torch.Tensor, iters: int = 20) -> float:
        return self.eng.bench_all_reduce(t, iters)

    def close(self):
        self.eng.shutdown()


NativeAllReduce = NativeComm  # name used by parallel.ddp
