"""Tracing and profiling hooks (SURVEY §5 "Tracing / profiling": the reference only had per-step
wall time in ``progress_bar`` and a tqdm rate — reference utils.py:68-75, main_dist.py:173).

* :func:`range_push` / :func:`range_pop` / :func:`trace_range` — ROCTX ranges (``libroctx64``,
  loaded with ctypes; no-ops when the library or ``PCA_ROCTX=0``), visible in
  ``rocprofv3 --marker-trace`` timelines. The trainer marks data / step / eval phases.
* :class:`StepTimer` — HIP-event step timing on the device's own clock (no host sync per step;
  ``summary()`` synchronises once).
* :func:`torch_profile` — a ``torch.profiler`` context (ROCm/roctracer activity) that writes a
  Chrome trace, used by ``--profile`` in main.py / main_dist.py.
* :func:`kernel_table` — per-kernel summary of a finished torch.profiler session.

For counter collection use ``rocprofv3 --kernel-trace --stats`` / ``--pmc`` from the outside
(tools/pmc_conv.sh, tools/prof_summary.py); nothing here changes the compute path.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time

import torch

_roctx = None
_roctx_tried = False


def _lib():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if os.environ.get("PCA_ROCTX", "1") == "0":
        return None
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    for name in (os.path.join(rocm, "lib", "libroctx64.so"), "libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


def roctx_available() -> bool:
    return _lib() is not None


def range_push(name: str) -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def range_pop() -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxRangePop()


def mark(name: str) -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def trace_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()


class StepTimer:
    """Device-side step timing with HIP events (CPU fallback: perf_counter)."""

    def __init__(self, device):
        self.cuda = torch.device(device).type == "cuda"
        self.events = []
        self.host = []

    def start(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events.append([e, None])
        else:
            self.host.append([time.perf_counter(), None])

    def stop(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events[-1][1] = e
        else:
            self.host[-1][1] = time.perf_counter()

    def times_ms(self):
        if self.cuda:
            torch.cuda.synchronize()
            return [a.elapsed_time(b) for a, b in self.events if b is not None]
        return [(b - a) * 1e3 for a, b in self.host if b is not None]

    def summary(self, skip: int = 0):
        t = sorted(self.times_ms()[skip:])
        if not t:
            return {}
        return {"steps": len(t), "mean_ms": sum(t) / len(t), "median_ms": t[len(t) // 2],
                "min_ms": t[0], "max_ms": t[-1]}


@contextlib.contextmanager
def torch_profile(trace_path: str | None, active: int = 5, warmup: int = 2):
    """torch.profiler over the enclosed steps; call ``prof.step()`` once per step."""
    from torch.profiler import ProfilerActivity, profile, schedule

    acts = [ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(ProfilerActivity.CUDA)

    def _done(p):
        if trace_path:
            os.makedirs(os.path.dirname(os.path.abspath(trace_path)), exist_ok=True)
            p.export_chrome_trace(trace_path)

    with profile(activities=acts, schedule=schedule(wait=0, warmup=warmup, active=active, repeat=1),
                 on_trace_ready=_done, record_shapes=False) as prof:
        yield prof


def kernel_table(prof, top: int = 25) -> str:
    key = "self_cuda_time_total" if torch.cuda.is_available() else "self_cpu_time_total"
    return prof.key_averages().table(sort_by=key, row_limit=top)
