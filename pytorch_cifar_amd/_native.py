"""Loader for the in-tree gfx950 kernel library.

GPU tensors always go through the native kernels: if the extension is missing on a machine with
a HIP device, ops raise instead of silently falling back to stock PyTorch kernels. CPU tensors use
the pure-PyTorch reference path (BASELINE config 1: LeNet on CPU).
"""
from __future__ import annotations

import os

_lib = None
_err: Exception | None = None


def lib():
    """Return the ``pytorch_cifar_amd._C`` module, building it in-tree on first use if needed."""
    global _lib, _err
    if _lib is not None:
        return _lib
    try:
        from . import _C  # noqa: F401

        _lib = _C
        return _lib
    except ImportError as e:  # not built yet
        _err = e
    if os.environ.get("PCA_NO_AUTOBUILD", "0") != "1":
        from . import _build

        _build.build()
        from . import _C  # noqa: F811

        _lib = _C
        return _lib
    raise RuntimeError(
        "pytorch_cifar_amd native extension is not built; run `python -m pytorch_cifar_amd._build`"
    ) from _err


def available() -> bool:
    try:
        lib()
        return True
    except Exception:
        return False


def loaded_path() -> str | None:
    return getattr(_lib, "__file__", None) if _lib is not None else None
