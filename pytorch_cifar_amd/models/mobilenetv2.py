"""MobileNetV2, CIFAR strides (parity: reference models/mobilenetv2.py:11-77).

Inverted residual: expand 1x1 (+BN+ReLU) -> depthwise 3x3 (+BN+ReLU) -> project 1x1 + BN, and
for stride 1 the residual (identity or 1x1 conv+BN) is folded into the projection BN pass. The
expand BN + ReLU is applied on the depthwise kernel's input loads (ops.functional.bn_act_dwconv):
the expanded activation is written once (pre-BN) instead of twice."""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F
from ._blocks import shortcut_kwargs


class Block(tnn.Module):
    """expand + depthwise + pointwise"""

    def __init__(self, in_planes, out_planes, expansion, stride):
        super().__init__()
        self.stride = stride
        planes = expansion * in_planes
        self.conv1 = Conv2d(in_planes, planes, kernel_size=1, stride=1, padding=0, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, groups=planes, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.conv3 = Conv2d(planes, out_planes, kernel_size=1, stride=1, padding=0, bias=False)
        self.bn3 = BatchNorm2d(out_planes)
        self.shortcut = Sequential()
        if stride == 1 and in_planes != out_planes:
            self.shortcut = Sequential(
                Conv2d(in_planes, out_planes, kernel_size=1, stride=1, padding=0, bias=False),
                BatchNorm2d(out_planes))

    def forward(self, x):
        # bn1 + ReLU applied inside the depthwise conv2's loads (its output is never written)
        out = F.bn_act_dwconv(self.bn1, self.conv1(x), "relu", self.conv2)
        out = self.bn2(out, act="relu")
        if self.stride == 1:
            return self.bn3(self.conv3(out), **shortcut_kwargs(self.shortcut, x))
        return self.bn3(self.conv3(out))


class MobileNetV2(tnn.Module):
    # (expansion, out_planes, num_blocks, stride); CIFAR: stride 1 in stage 2 and the stem
    cfg = [(1, 16, 1, 1),
           (6, 24, 2, 1),
           (6, 32, 3, 2),
           (6, 64, 4, 2),
           (6, 96, 3, 1),
           (6, 160, 3, 2),
           (6, 320, 1, 1)]

    def __init__(self, num_classes=10):
        super().__init__()
        self.conv1 = Conv2d(3, 32, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = BatchNorm2d(32)
        self.layers = self._make_layers(in_planes=32)
        self.conv2 = Conv2d(320, 1280, kernel_size=1, stride=1, padding=0, bias=False)
        self.bn2 = BatchNorm2d(1280)
        self.linear = Linear(1280, num_classes)

    def _make_layers(self, in_planes):
        layers = []
        for expansion, out_planes, num_blocks, stride in self.cfg:
            for s in [stride] + [1] * (num_blocks - 1):
                layers.append(Block(in_planes, out_planes, expansion, s))
                in_planes = out_planes
        return Sequential(*layers)

    def forward(self, x):
        out = self.layers(self.bn1(self.conv1(x), act="relu"))
        out = self.bn2(self.conv2(out), act="relu")
        return F.pool_linear(out, 4, self.linear)
