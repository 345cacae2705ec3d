"""EfficientNet-B0 for CIFAR (parity: reference models/efficientnet.py:12-164).

MBConv: expand 1x1 + BN + Swish (skipped when expand_ratio == 1 — its conv1/bn1 parameters still
exist, as in the reference, and never receive gradients; the data-parallel engine reduces them as
zeros), depthwise k3/k5 + BN + Swish, squeeze-excite with Swish, project 1x1 + BN (+ skip).
Drop-connect keeps the reference's schedule: ``b`` is never incremented (efficientnet.py:125,130),
so every rate is 0 and drop-connect never fires; final dropout 0.2 in training.
"""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F


def swish(x):
    return F.swish(x)


def drop_connect(x, drop_ratio, owner=None):
    """Per-sample drop-connect (efficientnet.py:16-22): native Philox keep byte per sample on the
    GPU (ops/functional.py drop_connect), Bernoulli mask on the CPU reference path. ``owner``
    (the block) holds the Philox state, so the trainer's state snapshot sees it."""
    return F.drop_connect(x, drop_ratio, owner=owner)


class SE(tnn.Module):
    """Squeeze-and-Excitation block with Swish."""

    def __init__(self, in_channels, se_channels):
        super().__init__()
        self.se1 = Conv2d(in_channels, se_channels, kernel_size=1, bias=True)
        self.se2 = Conv2d(se_channels, in_channels, kernel_size=1, bias=True)

    def forward(self, x):
        return F.se_gate(x, self.se1, self.se2, act="swish")


class Block(tnn.Module):
    """expansion + depthwise + pointwise + squeeze-excitation"""

    def __init__(self, in_channels, out_channels, kernel_size, stride, expand_ratio=1, se_ratio=0.0,
                 drop_rate=0.0):
        super().__init__()
        self.stride = stride
        self.drop_rate = drop_rate
        self.expand_ratio = expand_ratio
        channels = expand_ratio * in_channels
        self.conv1 = Conv2d(in_channels, channels, kernel_size=1, stride=1, padding=0, bias=False)
        self.bn1 = BatchNorm2d(channels)
        self.conv2 = Conv2d(channels, channels, kernel_size=kernel_size, stride=stride,
                            padding=(1 if kernel_size == 3 else 2), groups=channels, bias=False)
        self.bn2 = BatchNorm2d(channels)
        self.se = SE(channels, int(in_channels * se_ratio))
        self.conv3 = Conv2d(channels, out_channels, kernel_size=1, stride=1, padding=0, bias=False)
        self.bn3 = BatchNorm2d(out_channels)
        self.has_skip = (stride == 1) and (in_channels == out_channels)

    def forward(self, x):
        if self.expand_ratio == 1:
            out = self.bn2(self.conv2(x), act="swish")
        else:   # bn1 + swish applied inside the depthwise conv2's loads
            out = self.bn2(F.bn_act_dwconv(self.bn1, self.conv1(x), "swish", self.conv2), act="swish")
        out = self.se(out)
        y = self.conv3(out)
        if self.has_skip:
            if self.training and self.drop_rate > 0:
                return F.add_act(drop_connect(self.bn3(y), self.drop_rate, owner=self), x)
            return self.bn3(y, residual=x)
        return self.bn3(y)


class EfficientNet(tnn.Module):
    def __init__(self, cfg, num_classes=10):
        super().__init__()
        self.cfg = cfg
        self.conv1 = Conv2d(3, 32, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = BatchNorm2d(32)
        self.layers = self._make_layers(in_channels=32)
        self.linear = Linear(cfg["out_channels"][-1], num_classes)

    def _make_layers(self, in_channels):
        layers = []
        keys = ["expansion", "out_channels", "num_blocks", "kernel_size", "stride"]
        b = 0  # never incremented, exactly as the reference: all drop-connect rates are 0
        blocks = sum(self.cfg["num_blocks"])
        for expansion, out_channels, num_blocks, kernel_size, stride in zip(*[self.cfg[k] for k in keys]):
            for s in [stride] + [1] * (num_blocks - 1):
                drop_rate = self.cfg["drop_connect_rate"] * b / blocks
                layers.append(Block(in_channels, out_channels, kernel_size, s, expansion,
                                    se_ratio=0.25, drop_rate=drop_rate))
                in_channels = out_channels
        return Sequential(*layers)

    def forward(self, x):
        out = self.layers(self.bn1(self.conv1(x), act="swish"))
        # adaptive_avg_pool2d(1) -> flatten -> dropout(0.2, training) -> linear as one fused head
        # kernel each way (Philox keep mask; ops/functional.py pool_linear)
        return F.pool_linear(out, None, self.linear, self.cfg["dropout_rate"], self.training)


def EfficientNetB0():
    cfg = {
        "num_blocks": [1, 2, 2, 3, 3, 4, 1],
        "expansion": [1, 6, 6, 6, 6, 6, 6],
        "out_channels": [16, 24, 40, 80, 112, 192, 320],
        "kernel_size": [3, 3, 5, 3, 5, 5, 3],
        "stride": [1, 2, 2, 2, 1, 2, 1],
        "dropout_rate": 0.2,
        "drop_connect_rate": 0.2,
    }
    return EfficientNet(cfg)
