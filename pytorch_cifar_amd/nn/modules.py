"""Layer modules of the model zoo.

Subclasses of the torch.nn layers so parameter/buffer names, shapes, default initialisation and
``state_dict`` keys are exactly those of the reference models (``conv1.weight``,
``bn1.running_mean``, ``shortcut.0.weight`` ...), while ``forward`` routes through the fused
gfx950 ops of :mod:`pytorch_cifar_amd.ops.functional`:

* ``Conv2d`` keeps its weight channels_last (physically [Cout][KH][KW][Cin/G], the MFMA B
  operand) and, in training mode, asks the kernel for per-channel BatchNorm partial sums in its
  epilogue; they ride on the output tensor to the ``BatchNorm2d`` that consumes it.
* ``BatchNorm2d.forward(x, act=..., residual=..., residual_bn=...)`` is one fused
  normalize + residual + activation pass (plain ``bn(x)`` still works).
* ``Sequential`` fuses ``BatchNorm2d`` → ``ReLU`` pairs (the VGG/GoogLeNet/DLA stems).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops import functional as OF

_STATS_ATTR = "_pca_stats"


class Conv2d(nn.Conv2d):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        if self.dilation not in ((1, 1), 1):
            raise NotImplementedError("dilated convolutions are not used by the CIFAR zoo")
        if self.padding_mode != "zeros":
            raise NotImplementedError("only zero padding")
        with torch.no_grad():
            self.weight.data = self.weight.data.contiguous(memory_format=torch.channels_last)

    def forward(self, x, want_stats=None):
        if want_stats is None:
            want_stats = self.training
        want_stats = bool(want_stats and not OF._ref(x))
        acc = None
        # once a fusable BatchNorm consumed this conv's statistics (it sets _pca_acc_ok), they
        # travel through the conv's sharded accumulator instead of a slab (ops.functional.StatAcc)
        if want_stats and self.__dict__.get("_pca_acc_ok") and OF.acc_enabled(self.out_channels, x.device):
            acc = OF.stat_acc(self, "fwd", self.out_channels, 2, x.device)
        pilot = OF.conv_pilot(self, x.device) if want_stats else None
        brec = None
        if (self.bias is not None and self.bias.requires_grad and self.training
                and torch.is_grad_enabled() and not OF._ref(x)):
            brec = OF.BiasRec(self.bias)
        y, stats = OF.conv2d(x, self.weight, self.bias, self.stride, self.padding, self.groups,
                             want_stats, acc, pilot, brec)
        if brec is not None:
            y._pca_bias_rec = brec
        if stats is not None:
            setattr(y, _STATS_ATTR, stats)
            y._pca_stats_src = self
        elif want_stats and self.groups > 1 and self.groups == self.in_channels and \
                self.bias is None:
            # depthwise: no statistics until a fusable BN accepts them (it sets _pca_acc_ok); from
            # then on the kernel adds them into the accumulator this module passes
            y._pca_stats_src = self
        return y

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)
        # load_state_dict copies values into the existing (channels_last) storage; nothing else
        # to do, but keep the layout invariant explicit for parameters replaced wholesale.
        if not self.weight.is_contiguous(memory_format=torch.channels_last):
            with torch.no_grad():
                self.weight.data = self.weight.data.contiguous(memory_format=torch.channels_last)


class BatchNorm2d(nn.BatchNorm2d):
    def forward(self, x, act=None, residual=None, residual_bn=None, out=None):
        """``out``: a ChannelSlab destination slice (zero-copy concatenation), GPU path only."""
        stats = getattr(x, _STATS_ATTR, None) if self.training else None
        rb = None
        if residual_bn is not None:
            bn_b, xb = residual_bn
            rb = (bn_b, xb, getattr(xb, _STATS_ATTR, None) if bn_b.training else None)
        return OF.batch_norm_act(self, x, act, residual, rb, stats, out=out)


class Linear(nn.Linear):
    def forward(self, x):
        if x.dtype != self.weight.dtype:
            x = x.to(self.weight.dtype)
        return nn.functional.linear(x, self.weight, self.bias)


class ReLU(nn.ReLU):
    def forward(self, x):
        return OF.relu(x)


class MaxPool2d(nn.MaxPool2d):
    def forward(self, x):
        return OF.max_pool2d(x, self.kernel_size, self.stride, self.padding)


class AvgPool2d(nn.AvgPool2d):
    def forward(self, x):
        return OF.avg_pool2d(x, self.kernel_size, self.stride, self.padding)


class Sequential(nn.Sequential):
    """nn.Sequential that fuses BatchNorm2d -> ReLU into one kernel pass.

    ``out`` (a ChannelSlab destination slice): the final BatchNorm(+ReLU) writes its result there
    (zero-copy concatenation, googlenet.py Inception); a Sequential not ending in one cannot."""

    def forward(self, x, out=None):
        mods = list(self._modules.values())
        i = 0
        while i < len(mods):
            m = mods[i]
            if isinstance(m, BatchNorm2d) and i + 1 < len(mods) and isinstance(mods[i + 1], (ReLU, nn.ReLU)):
                last = i + 2 == len(mods)
                x = m(x, act="relu", out=out if last else None)
                i += 2
                continue
            if out is not None and i + 1 == len(mods):
                if not isinstance(m, BatchNorm2d):
                    raise ValueError("Sequential(out=...) needs a final BatchNorm2d(+ReLU)")
                x = m(x, out=out)
                i += 1
                continue
            x = m(x)
            if (isinstance(m, Conv2d) and m.bias is not None and i + 1 < len(mods)
                    and isinstance(mods[i + 1], BatchNorm2d)):
                # only the next BatchNorm reads this conv output: its backward may deliver the
                # conv's bias gradient (ops.functional.BiasRec)
                x._pca_bias_sole = True
            i += 1
        return x

    def ends_in_bn(self):
        mods = list(self._modules.values())
        return bool(mods) and (isinstance(mods[-1], BatchNorm2d) or
                               (len(mods) > 1 and isinstance(mods[-2], BatchNorm2d) and
                                isinstance(mods[-1], (ReLU, nn.ReLU))))
