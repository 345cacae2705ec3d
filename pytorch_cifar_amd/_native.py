"""Loader for the in-tree gfx950 kernel library.

GPU tensors always go through the native kernels: if the extension is missing on a machine with
a HIP device, ops raise instead of silently falling back to stock PyTorch kernels. CPU tensors use
the pure-PyTorch reference path (BASELINE config 1: LeNet on CPU).

Debug mode (SURVEY §5 race/fault detection): with ``PCA_DEBUG_SYNC=1`` (or
:func:`set_debug_sync`) every native entry point is followed by a device synchronisation and a
``hipGetLastError`` check, so an asynchronous kernel fault or launch error is raised at the op that
caused it (named in the message) instead of at some later sync point — the HIP analogue of
``CUDA_LAUNCH_BLOCKING=1`` scoped to this library.
"""
from __future__ import annotations

import os
import sys

_lib = None
_err: Exception | None = None
_debug = os.environ.get("PCA_DEBUG_SYNC", "0") == "1"
_trace = os.environ.get("PCA_DEBUG_TRACE", "0") == "1"


class _DebugProxy:
    """Wraps the extension: sync + error check after every call (debug mode only)."""

    def __init__(self, mod):
        self._mod = mod
        self.__file__ = getattr(mod, "__file__", None)

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn) or isinstance(fn, type) or name in ("last_error",):
            return fn

        def wrapped(*a, **k):
            import torch

            if _trace:   # PCA_DEBUG_TRACE=1: name every op before it runs (a device fault that
                         # aborts the process then has its op on the last stderr line)
                import sys

                shapes = [tuple(x.shape) for x in a if hasattr(x, "shape")][:4]
                print(f"[native] {name} {shapes}", file=sys.stderr, flush=True)
            out = fn(*a, **k)
            err = self._mod.last_error()
            if err:
                raise RuntimeError(f"pytorch_cifar_amd._C.{name}: launch failed: {err}")
            if torch.cuda.is_available():
                try:
                    torch.cuda.synchronize()
                except Exception as e:  # device fault surfaced by this op
                    raise RuntimeError(f"pytorch_cifar_amd._C.{name}: device error: {e}") from e
            return out

        return wrapped


def set_debug_sync(on: bool = True) -> None:
    global _debug
    _debug = bool(on)


def _wrap(mod):
    return _DebugProxy(mod) if _debug else mod


def lib():
    """Return the ``pytorch_cifar_amd._C`` module, building it in-tree on first use if needed."""
    global _lib, _err
    if _lib is not None:
        return _wrap(_lib)
    from . import _build

    # torch first: its libamdhip64 / librccl (SONAME .so.7 / .so.1) then satisfy _C's NEEDED
    # entries. Loading _C first pulls /opt/rocm's copies in as well — two HIP runtimes and two
    # RCCLs in one process, whose exit-time destructors corrupt the heap.
    import torch  # noqa: F401

    stale = _build.is_stale()
    no_build = os.environ.get("PCA_NO_AUTOBUILD", "0") == "1"
    if stale or (stale is None and not no_build):
        # the .so is missing or was built from other csrc contents: never run a stale kernel
        # library silently (a stale .so ships with the tree to the GPU box)
        if no_build:
            raise RuntimeError(
                "pytorch_cifar_amd native extension is missing or stale (csrc changed since it was "
                "built); run `python -m pytorch_cifar_amd._build`")
        _build.build_locked()
    try:
        from . import _C  # noqa: F401

        if stale is None and no_build:
            # no recorded digest next to the .so: trust the one it carries
            want = _build.source_digest()
            have = _C.src_digest() if hasattr(_C, "src_digest") else None
            if have != want:
                raise RuntimeError(
                    "pytorch_cifar_amd native extension was built from other sources "
                    f"(digest {have} != {want}); run `python -m pytorch_cifar_amd._build`")
            import warnings

            warnings.warn("pytorch_cifar_amd: .srchash missing; the .so's embedded source digest matches")
        _lib = _C
        _tune_cache(_lib)
        return _wrap(_lib)
    except ImportError as e:  # not built yet
        _err = e
    if os.environ.get("PCA_NO_AUTOBUILD", "0") != "1":
        _build.build_locked(force=True)
        from . import _C  # noqa: F811

        _lib = _C
        _tune_cache(_lib)
        return _wrap(_lib)
    raise RuntimeError(
        "pytorch_cifar_amd native extension is not built; run `python -m pytorch_cifar_amd._build`"
    ) from _err


def _tune_cache(mod):
    """Kernel selection at load: the shipped MI355X tune table (engine/tuning.py; PCA_TUNE_TABLE=0
    skips it), then PCA_TUNE_CACHE=<file.json>: restore the conv autotuner's choices at load and
    save them at exit (the reference's cudnn.benchmark re-times every run; here a cache skips the
    trials, and profiled runs reuse the choices an un-profiled run made)."""
    try:
        from .engine.tuning import load_table

        load_table(mod)
    except Exception as e:    # a bad table must not stop the library loading: say why, tune afresh
        print(f"pytorch_cifar_amd: shipped tune table failed to load ({type(e).__name__}: {e})",
              file=sys.stderr)
    path = os.environ.get("PCA_TUNE_CACHE")
    if not path or not hasattr(mod, "tune_import"):
        return
    import atexit
    import json

    try:
        with open(path) as fh:
            mod.tune_import(json.load(fh))
    except (OSError, ValueError):
        pass

    def save():
        try:
            rows = mod.tune_export()
            if not rows:
                return
            tmp = f"{path}.{os.getpid()}.tmp"
            with open(tmp, "w") as fh:
                json.dump(rows, fh)
            os.replace(tmp, path)
        except Exception:
            pass

    atexit.register(save)


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def loaded_path() -> str | None:
    return getattr(_lib, "__file__", None) if _lib is not None else None
