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


def free_port(host: str = "127.0.0.1") -> int:
    import socket

    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def spawned_world() -> int:
    """WORLD_SIZE of the torchrun-style environment (0 when this process was not launched as a rank)."""
    return int(os.environ.get("WORLD_SIZE", "0") or 0)


def spawn_local_ranks(nprocs: int, argv: list[str], env_extra: dict | None = None,
                      poll_s: float = 0.2) -> int:
    """Run ``python argv...`` as ``nprocs`` rank processes of one node and wait for them.

    The self-contained equivalent of ``torchrun --nnodes 1 --nproc-per-node N`` / the reference's
    ``mp.spawn(main_worker, nprocs=ngpus)`` (main_dist.py:51-60): each child gets the torchrun env
    (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT) and
    binds GPU LOCAL_RANK in :func:`init_from_env`. The parent never touches the GPU (it must not:
    children are started as fresh interpreters, never by exec'ing a process that initialised HIP),
    forwards SIGINT/SIGTERM, and if any rank fails it terminates the others (exact child PIDs)
    so a collective blocked on the dead rank cannot hang the job. Returns the first non-zero exit
    code (0 when every rank succeeded).
    """
    import signal
    import subprocess
    import sys
    import time

    port = free_port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC (RCCL peer buffers)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nprocs),
                    "LOCAL_WORLD_SIZE": str(nprocs), "GROUP_RANK": "0",
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        env.update(env_extra or {})
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env))

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except ProcessLookupError:
                    pass

    prev = {}
    for s in (signal.SIGINT, signal.SIGTERM):
        try:
            prev[s] = signal.signal(s, lambda sig, _f: stop_all(sig))
        except ValueError:        # not the main thread
            pass
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                stop_all()
                deadline = time.time() + 30
                for p in procs:
                    try:
                        p.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        p.kill()
                        p.wait()
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        for s, h in prev.items():
            signal.signal(s, h)
    return rc


def init_from_env(backend: str = "nccl", native_comm: bool = True) -> DistContext:
    """Initialise from torchrun-style environment variables (single process if absent)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    return init_distributed(rank, world, local_rank, backend=backend, native_comm=native_comm)
