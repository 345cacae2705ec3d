"""RegNetX_200MF / RegNetX_400MF / RegNetY_400MF (parity: reference models/regnet.py:12-143).

X: 1x1 -> grouped 3x3 (group width 8/16, i.e. 3..46 groups) -> 1x1 with projection shortcut;
Y adds squeeze-excitation (ReLU) after the grouped conv. Grouped convs with 8- or 16-channel
groups run on the MFMA kernel, one GEMM per group along grid.z."""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F
from ._blocks import shortcut_kwargs


class SE(tnn.Module):
    """Squeeze-and-Excitation block."""

    def __init__(self, in_planes, se_planes):
        super().__init__()
        self.se1 = Conv2d(in_planes, se_planes, kernel_size=1, bias=True)
        self.se2 = Conv2d(se_planes, in_planes, kernel_size=1, bias=True)

    def forward(self, x):
        return F.se_gate(x, self.se1, self.se2, act="relu")


class Block(tnn.Module):
    def __init__(self, w_in, w_out, stride, group_width, bottleneck_ratio, se_ratio):
        super().__init__()
        w_b = int(round(w_out * bottleneck_ratio))
        self.conv1 = Conv2d(w_in, w_b, kernel_size=1, bias=False)
        self.bn1 = BatchNorm2d(w_b)
        num_groups = w_b // group_width
        self.conv2 = Conv2d(w_b, w_b, kernel_size=3, stride=stride, padding=1, groups=num_groups, bias=False)
        self.bn2 = BatchNorm2d(w_b)
        self.with_se = se_ratio > 0
        if self.with_se:
            self.se = SE(w_b, int(round(w_in * se_ratio)))
        self.conv3 = Conv2d(w_b, w_out, kernel_size=1, bias=False)
        self.bn3 = BatchNorm2d(w_out)
        self.shortcut = Sequential()
        if stride != 1 or w_in != w_out:
            self.shortcut = Sequential(
                Conv2d(w_in, w_out, kernel_size=1, stride=stride, bias=False), BatchNorm2d(w_out))

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.bn2(self.conv2(out), act="relu")
        if self.with_se:
            out = self.se(out)
        return self.bn3(self.conv3(out), act="relu", **shortcut_kwargs(self.shortcut, x))


class RegNet(tnn.Module):
    def __init__(self, cfg, num_classes=10):
        super().__init__()
        self.cfg = cfg
        self.in_planes = 64
        self.conv1 = Conv2d(3, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.layer1 = self._make_layer(0)
        self.layer2 = self._make_layer(1)
        self.layer3 = self._make_layer(2)
        self.layer4 = self._make_layer(3)
        self.linear = Linear(self.cfg["widths"][-1], num_classes)

    def _make_layer(self, idx):
        c = self.cfg
        layers = []
        for i in range(c["depths"][idx]):
            s = c["strides"][idx] if i == 0 else 1
            layers.append(Block(self.in_planes, c["widths"][idx], s, c["group_width"],
                                c["bottleneck_ratio"], c["se_ratio"]))
            self.in_planes = c["widths"][idx]
        return Sequential(*layers)

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.layer4(self.layer3(self.layer2(self.layer1(out))))
        return F.pool_linear(out, None, self.linear)


def RegNetX_200MF():
    return RegNet({"depths": [1, 1, 4, 7], "widths": [24, 56, 152, 368], "strides": [1, 1, 2, 2],
                   "group_width": 8, "bottleneck_ratio": 1, "se_ratio": 0})


def RegNetX_400MF():
    return RegNet({"depths": [1, 2, 7, 12], "widths": [32, 64, 160, 384], "strides": [1, 1, 2, 2],
                   "group_width": 16, "bottleneck_ratio": 1, "se_ratio": 0})


def RegNetY_400MF():
    return RegNet({"depths": [1, 2, 7, 12], "widths": [32, 64, 160, 384], "strides": [1, 1, 2, 2],
                   "group_width": 16, "bottleneck_ratio": 1, "se_ratio": 0.25})
