"""Dual Path Networks DPN26 / DPN92 (parity: reference models/dpn.py:7-89).

Bottleneck: 1x1 -> grouped 3x3 (32 groups, 3..24 channels per group: direct-conv kernel) -> 1x1,
then the dual path: residual-add of the first ``out_planes`` channels and dense concatenation of
the rest, followed by ReLU — one native pass each way (``F.dpn_merge``)."""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F


class Bottleneck(tnn.Module):
    def __init__(self, last_planes, in_planes, out_planes, dense_depth, stride, first_layer):
        super().__init__()
        self.out_planes = out_planes
        self.dense_depth = dense_depth
        self.conv1 = Conv2d(last_planes, in_planes, kernel_size=1, bias=False)
        self.bn1 = BatchNorm2d(in_planes)
        self.conv2 = Conv2d(in_planes, in_planes, kernel_size=3, stride=stride, padding=1, groups=32, bias=False)
        self.bn2 = BatchNorm2d(in_planes)
        self.conv3 = Conv2d(in_planes, out_planes + dense_depth, kernel_size=1, bias=False)
        self.bn3 = BatchNorm2d(out_planes + dense_depth)
        self.shortcut = Sequential()
        if first_layer:
            self.shortcut = Sequential(
                Conv2d(last_planes, out_planes + dense_depth, kernel_size=1, stride=stride, bias=False),
                BatchNorm2d(out_planes + dense_depth))

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.bn2(self.conv2(out), act="relu")
        out = self.bn3(self.conv3(out))
        x = self.shortcut(x)
        return F.dpn_merge(x, out, self.out_planes)


class DPN(tnn.Module):
    def __init__(self, cfg):
        super().__init__()
        in_planes, out_planes = cfg["in_planes"], cfg["out_planes"]
        num_blocks, dense_depth = cfg["num_blocks"], cfg["dense_depth"]
        self.conv1 = Conv2d(3, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.last_planes = 64
        self.layer1 = self._make_layer(in_planes[0], out_planes[0], num_blocks[0], dense_depth[0], stride=1)
        self.layer2 = self._make_layer(in_planes[1], out_planes[1], num_blocks[1], dense_depth[1], stride=2)
        self.layer3 = self._make_layer(in_planes[2], out_planes[2], num_blocks[2], dense_depth[2], stride=2)
        self.layer4 = self._make_layer(in_planes[3], out_planes[3], num_blocks[3], dense_depth[3], stride=2)
        self.linear = Linear(out_planes[3] + (num_blocks[3] + 1) * dense_depth[3], 10)

    def _make_layer(self, in_planes, out_planes, num_blocks, dense_depth, stride):
        layers = []
        for i, s in enumerate([stride] + [1] * (num_blocks - 1)):
            layers.append(Bottleneck(self.last_planes, in_planes, out_planes, dense_depth, s, i == 0))
            self.last_planes = out_planes + (i + 2) * dense_depth
        return Sequential(*layers)

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.layer4(self.layer3(self.layer2(self.layer1(out))))
        return F.pool_linear(out, 4, self.linear)


def DPN26():
    return DPN({"in_planes": (96, 192, 384, 768), "out_planes": (256, 512, 1024, 2048),
                "num_blocks": (2, 2, 2, 2), "dense_depth": (16, 32, 24, 128)})


def DPN92():
    return DPN({"in_planes": (96, 192, 384, 768), "out_planes": (256, 512, 1024, 2048),
                "num_blocks": (3, 4, 20, 3), "dense_depth": (16, 32, 24, 128)})
