"""Process-group bootstrap: one process per GPU, rendezvous from the env the training operator
(or torchrun) injects -- ``MASTER_ADDR/MASTER_PORT/WORLD_SIZE/RANK/LOCAL_RANK``
(reference injects only ``NCCL_DEBUG`` at
``/root/reference/app/jobs/kubeflow/PyTorchJobDeployer.py:115``).

On ROCm the ``nccl`` backend of torch.distributed IS RCCL; collectives run over xGMI inside a node.
CPU runs (tests, the CPU plumbing job) use ``gloo``.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


def init_distributed(device_type: str = "auto", timeout_s: int = 1800) -> DistInfo:
    """Initialise torch.distributed when WORLD_SIZE > 1; bind this rank to its GPU.

    ``FTC_COLLECTIVE_TIMEOUT_S`` overrides ``timeout_s``: a collective a lost peer never joins aborts
    the rank (RCCL watchdog) or raises (gloo) after that long, so the job fails over to its restart
    path instead of holding its GPUs (``utils.faults``)."""
    timeout_s = int(float(os.environ.get("FTC_COLLECTIVE_TIMEOUT_S") or timeout_s))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device_type == "auto":
        # device_count() does not initialise the HIP runtime on this image; is_available() does
        device_type = "cuda" if torch.cuda.device_count() > 0 and torch.cuda.is_available() else "cpu"
    share = os.environ.get("FTC_SHARE_GPU") == "1"
    if device_type == "cuda":
        # FTC_SHARE_GPU=1: several ranks on one card (rehearsing the multi-GPU path on a 1-GPU box)
        idx = local_device_index(local, torch.cuda.device_count(), share)
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    backend = "none"
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        # nccl (= RCCL over xGMI) for GPU ranks; FTC_DIST_BACKEND=gloo forces host collectives (CPU
        # tests, shared-card rehearsals where RCCL refuses two ranks on one device)
        backend = os.environ.get("FTC_DIST_BACKEND") or ("nccl" if device.type == "cuda" else "gloo")
        if backend == "nccl" and os.environ.get("FTC_SHARE_GPU") == "1":
            # rehearsal of the multi-GPU RCCL path on ONE card: RCCL refuses two ranks on one device of
            # one host ("Duplicate GPU detected"), so every rank claims its own host id -- RCCL then
            # connects them through its socket transport over loopback.  Never set on a real node.
            os.environ.setdefault("NCCL_HOSTID", f"ftc-rehearsal-rank{rank}")
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            os.environ.setdefault("NCCL_IB_DISABLE", "1")
        if not dist.is_initialized():
            kw = {}
            if backend == "nccl":
                kw["device_id"] = device
            # FTC_INIT_METHOD (e.g. file://...) overrides the env:// TCPStore rendezvous; tests use it
            dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                    init_method=os.environ.get("FTC_INIT_METHOD") or None,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        if device.type == "cuda" and not share:
            # one GPU per rank: a weak-scaling number from ranks sharing a card would be mislabelled
            import socket

            me = (socket.gethostname(), device_key(device), rank)
            allr: list = [None] * world
            dist.all_gather_object(allr, me)
            check_distinct_devices(allr)
    return DistInfo(rank, world, local, backend, device)


def device_key(device: torch.device) -> str:
    """A host-unique id of the physical GPU: its PCI domain:bus:device when the runtime reports one (never
    shared by two cards, whatever HIP_VISIBLE_DEVICES each rank got), plus the UUID -- a UUID alone is not
    trusted to differ between cards (some virtualised / containerised setups report one value for all)."""
    props = torch.cuda.get_device_properties(device)
    pci = [getattr(props, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id")]
    uuid = str(getattr(props, "uuid", "") or "")
    if all(v is not None for v in pci):
        return "pci:%x:%x:%x/%s" % (pci[0], pci[1], pci[2], uuid)
    return uuid or f"index{device.index}"


def local_device_index(local: int, count: int, share: bool = False) -> int:
    """The visible-device index this rank binds to: ``LOCAL_RANK`` when every rank sees the node's GPUs
    (torchrun), device 0 when the launcher narrowed each rank to ONE visible device (a per-rank
    ``HIP_VISIBLE_DEVICES``; the distinct-device check after the rendezvous still refuses two ranks on
    one card), ``LOCAL_RANK mod count`` for a shared-card rehearsal."""
    if share:
        return local % count
    if count == 1 and _narrowed_to_one_device():
        return 0
    check_local_rank(local, count)
    return local


def _narrowed_to_one_device() -> bool:
    """True when this rank's single visible device is its own: the launcher narrowed the visible set
    (``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``), or the node runs one
    rank (``LOCAL_WORLD_SIZE`` 1).  ``torchrun --nproc-per-node 2`` on a one-GPU host is neither, and gets
    the clear ``LOCAL_RANK`` error before the rendezvous instead of RCCL's 'Duplicate GPU' after it."""
    if any(os.environ.get(k, "").strip() for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES",
                                                    "CUDA_VISIBLE_DEVICES")):
        return True
    return int(os.environ.get("LOCAL_WORLD_SIZE", "1") or "1") == 1


def check_local_rank(local: int, count: int) -> None:
    if local >= count:
        raise RuntimeError(f"LOCAL_RANK {local} has no GPU of its own: {count} visible device(s) "
                           "(set FTC_SHARE_GPU=1 only to rehearse several ranks on one card)")


def check_distinct_devices(entries) -> None:
    """``entries``: (host, device id, rank) of every rank.  Two ranks of one host on one device raise."""
    seen: dict = {}
    for host, dev, rank in entries:
        other = seen.setdefault((host, dev), rank)
        if other != rank:
            raise RuntimeError(f"ranks {other} and {rank} are bound to the same GPU ({dev}) on {host}; "
                               "each rank needs its own device (FTC_SHARE_GPU=1 to rehearse on one card)")


def barrier(info: DistInfo):
    if info.distributed:
        if info.backend == "nccl":
            dist.barrier(device_ids=[info.device.index])
        else:
            dist.barrier()


def all_reduce_max(x: float, info: DistInfo) -> float:
    if not info.distributed:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=info.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_mean_(t: torch.Tensor, info: DistInfo) -> torch.Tensor:
    if info.distributed:
        dist.all_reduce(t)
        t /= info.world_size
    return t


def broadcast_params_(params, info: DistInfo, src: int = 0):
    """Make every rank start from rank 0's weights (N2 in SURVEY.md §2.3)."""
    if not info.distributed:
        return
    for p in params:
        dist.broadcast(p.data, src=src)


_TENSOR = "__ftc_tensor__"


def broadcast_state(obj, info: DistInfo, src: int = 0):
    """Broadcast a nested dict / list of CPU tensors and plain values from rank ``src``; every rank
    returns the same structure with CPU tensors.

    The resume path of ranks that cannot read ``src``'s checkpoint file (pod-local volumes of a
    multi-node job).  The structure travels pickled once (``broadcast_object_list`` -- our own state,
    rank to rank); each tensor is one broadcast on the group's device, so a full fine-tune's
    optimizer state never has to exist as a single pickled blob."""
    if not info.distributed:
        return obj
    tensors = []

    def skel(o):
        if torch.is_tensor(o):
            tensors.append(o)
            return (_TENSOR, len(tensors) - 1, tuple(o.shape), o.dtype)
        if isinstance(o, dict):
            return {k: skel(v) for k, v in o.items()}
        if isinstance(o, (list, tuple)):
            return type(o)(skel(v) for v in o)
        return o

    box = [skel(obj) if info.rank == src else None]
    dist.broadcast_object_list(box, src=src, device=info.device if info.backend == "nccl" else None)
    dev = info.device if info.backend == "nccl" else torch.device("cpu")

    def fill(o):
        if isinstance(o, tuple) and len(o) == 4 and o[0] == _TENSOR:
            _, i, shape, dtype = o
            if info.rank == src:
                t = tensors[i].detach().to(dev).contiguous()
            else:
                t = torch.empty(shape, dtype=dtype, device=dev)
            dist.broadcast(t, src=src)
            return t.cpu()
        if isinstance(o, dict):
            return {k: fill(v) for k, v in o.items()}
        if isinstance(o, (list, tuple)):
            return type(o)(fill(v) for v in o)
        return o

    return fill(box[0])


def destroy(info: DistInfo):
    if info.distributed and dist.is_initialized():
        dist.destroy_process_group()
