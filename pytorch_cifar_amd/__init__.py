"""pytorch_cifar_amd — an MI355X-native (gfx950 / CDNA4) CIFAR-10 training framework with the
capabilities of kuangliu-style pytorch-cifar (reference: aqualovers/pytorch-cifar).

Layers (re-designed MI355X-first):
  csrc/      hand-written HIP kernels (MFMA implicit-GEMM convs, halo wgrad, fused BN/act, CE,
             SGD, pools, depthwise, augmentation) + the native RCCL communicator
  ops/       autograd functions over the kernels (CPU tensors take a pure-PyTorch reference path)
  nn/        drop-in modules (Conv2d / BatchNorm2d / Linear ...) with reference state_dict layout
  models/    the full model zoo (44 configurations)
  engine/    flat parameter arena, SGD, hipGraph train step, trainer, checkpoints
  parallel/  process launcher, bucketed RCCL DDP, DataParallel
  data/      CIFAR-10 readers, synthetic data, GPU-resident loader with on-device augmentation
  utils/     reference-compatible helpers, profiling / ROCTX tracing
"""
from __future__ import annotations

__version__ = "0.1.0"


def set_deterministic(on: bool = True) -> None:
    """Bitwise-reproducible training: weight gradients are reduced through ordered slab rows
    instead of fp32 atomics (all other native kernels are already order-deterministic)."""
    from . import _native
    from .ops import functional

    _native.lib().set_deterministic(bool(on))
    functional.set_deterministic_flag(on)


def set_debug_sync(on: bool = True) -> None:
    """Synchronise and error-check after every native op (see ``_native`` debug mode)."""
    from . import _native

    _native.set_debug_sync(on)
