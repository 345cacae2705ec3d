"""Process-group bootstrap: one process per GPU (torchrun env or mp.spawn), RCCL over xGMI.

Replaces main_dist.py:51-82 (``mp.spawn`` + ``init_process_group('nccl', tcp://...)`` +
``set_device`` + ``barrier``).  On ROCm the "nccl" backend of torch.distributed *is* RCCL; in
addition every GPU rank owns a native :class:`pytorch_cifar_amd._C.RcclComm` (created from a
unique id exchanged through the process group) that the data-parallel engine drives directly on
its own HIP stream.  CPU-only runs (tests) use gloo and the torch.distributed collectives.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    backend: str = "none"
    comm: object = None  # native RcclComm on GPU ranks (world > 1)

    @property
    def distributed(self) -> bool:
        return self.world > 1

    def barrier(self):
        if self.distributed:
            if self.device.type == "cuda":
                dist.barrier(device_ids=[self.device.index])
            else:
                dist.barrier()

    def all_reduce_max(self, t: torch.Tensor) -> torch.Tensor:
        if self.distributed:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        if self.distributed:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t

    def health_check(self):
        """Raise if the native RCCL communicator reports an asynchronous error (failure
        detection); the communicator is aborted first so peers blocked in a
        collective are released instead of hanging until the process-group timeout."""
        if self.comm is None:
            return
        err = self.comm.async_error()
        if err:
            try:
                self.comm.abort()
            finally:
                self.comm = None
            raise RuntimeError(f"RCCL communicator error on rank {self.rank}: {err}")

    def shutdown(self):
        if self.comm is not None:
            try:
                self.comm.destroy()
            except Exception:
                pass
            self.comm = None
        if self.distributed and dist.is_initialized():
            dist.destroy_process_group()


def _make_native_comm(rank, world, device):
    from .. import _native

    C = _native.lib()
    obj = [C.rccl_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return C.RcclComm(obj[0], world, rank, device.index)


def init_distributed(rank: int, world: int, local_rank: int, backend: str = "nccl",
                     init_method: str | None = None, timeout_s: float = 600.0,
                     native_comm: bool = True) -> DistContext:
    use_cuda = torch.cuda.is_available() and backend != "gloo"
    if use_cuda:
        device = torch.device("cuda", local_rank)
        torch.cuda.set_device(device)
    else:
        device = torch.device("cpu")
        backend = "gloo"
    ctx = DistContext(rank=rank, world=world, local_rank=local_rank, device=device, backend=backend)
    if world > 1:
        kw = dict(backend=backend, world_size=world, rank=rank,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if init_method:
            kw["init_method"] = init_method
        if use_cuda:
            kw["device_id"] = device
        dist.init_process_group(**kw)
        if use_cuda and native_comm:
            ctx.comm = _make_native_comm(rank, world, device)
    return ctx


def init_from_env(backend: str = "nccl", native_comm: bool = True) -> DistContext:
    """Initialise from torchrun-style environment variables (single process if absent)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    return init_distributed(rank, world, local_rank, backend=backend, native_comm=native_comm)
