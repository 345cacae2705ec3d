"""Direct gradient delivery for native backward kernels.

The native backward passes write parameter gradients straight into ``param.grad`` (the wgrad
kernel accumulates with fp32 atomics, the BN finalize kernel adds in place) instead of returning
them through autograd's AccumulateGrad. That keeps the gradient buffers at fixed addresses (flat
gradient arena, hipGraph replay, RCCL buckets that are views of the arena) and saves one
read-modify-write pass per parameter. Because AccumulateGrad is bypassed, ``post_accumulate_grad``
hooks do not fire for these parameters; consumers (the data-parallel engine) register through
:func:`register_grad_ready_hook`, which covers both delivery paths.
"""
from __future__ import annotations

from typing import Callable

import torch

_HOOK_ATTR = "_pca_grad_ready_hooks"


def physical(p: torch.Tensor) -> torch.Tensor:
    """View of ``p`` in its physical memory order.

    4-D conv weights are kept channels_last, i.e. physically [Cout][KH][KW][Cin/G] — the
    K-contiguous GEMM operand of the MFMA kernels.  Everything else is plain contiguous.
    """
    if p.dim() == 4:
        v = p.permute(0, 2, 3, 1)
        if v.is_contiguous():
            return v
    return p


def grad_buffer(p: torch.Tensor) -> torch.Tensor | None:
    """Return ``p.grad`` in physical order if it can be accumulated into in place.

    Creates a zeroed gradient with the parameter's strides when ``p.grad`` is None. Returns None
    when the existing gradient has an incompatible layout (caller then adds a temporary).
    """
    if p.grad is None:
        p.grad = torch.zeros_like(p, memory_format=torch.preserve_format)
    g = p.grad
    if g.dtype != torch.float32:
        return None
    if p.dim() == 4:
        v = g.permute(0, 2, 3, 1)
        return v if v.is_contiguous() else None
    return g if g.is_contiguous() else None


def accumulate(p: torch.Tensor, g_phys: torch.Tensor) -> None:
    """Add a gradient given in physical order into ``p.grad`` and fire the ready hooks."""
    buf = grad_buffer(p)
    if buf is not None:
        if buf.data_ptr() != g_phys.data_ptr():
            buf.add_(g_phys.view_as(buf))
    else:
        if p.dim() == 4 and g_phys.dim() == 4:
            p.grad.add_(g_phys.permute(0, 3, 1, 2))
        else:
            p.grad.add_(g_phys.view_as(p.grad))
    fire(p)


def fire(p: torch.Tensor) -> None:
    for h in getattr(p, _HOOK_ATTR, ()):
        h(p)


def register_grad_ready_hook(p: torch.Tensor, fn: Callable[[torch.Tensor], None]):
    """Call ``fn(p)`` whenever a gradient for ``p`` has been delivered (either path)."""
    hooks = getattr(p, _HOOK_ATTR, None)
    if hooks is None:
        hooks = []
        setattr(p, _HOOK_ATTR, hooks)
    hooks.append(fn)
    handle = p.register_post_accumulate_grad_hook(fn)
    return handle


def clear_grad_ready_hooks(p: torch.Tensor) -> None:
    if hasattr(p, _HOOK_ATTR):
        delattr(p, _HOOK_ATTR)
