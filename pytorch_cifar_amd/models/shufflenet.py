"""ShuffleNetG2/G3 (parity: reference models/shufflenet.py:10-100).

The reference cannot construct these under Python 3 (``mid_planes = out_planes/4`` is a float,
shufflenet.py:27 — SURVEY App. B #3); here it is ``out_planes // 4``, everything else unchanged:
grouped 1x1 -> channel shuffle -> depthwise 3x3 -> grouped 1x1, with an AvgPool2d(3, 2, 1)
shortcut concatenated at stride 2 and added otherwise."""
import torch.nn as tnn

from ..nn import AvgPool2d, BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F


class ShuffleBlock(tnn.Module):
    def __init__(self, groups):
        super().__init__()
        self.groups = groups

    def forward(self, x):
        """Channel shuffle: [N,C,H,W] -> [N,g,C/g,H,W] -> [N,C/g,g,H,W] -> [N,C,H,W]"""
        return F.channel_shuffle(x, self.groups)


class Bottleneck(tnn.Module):
    def __init__(self, in_planes, out_planes, stride, groups):
        super().__init__()
        self.stride = stride
        mid_planes = out_planes // 4
        g = 1 if in_planes == 24 else groups
        self.conv1 = Conv2d(in_planes, mid_planes, kernel_size=1, groups=g, bias=False)
        self.bn1 = BatchNorm2d(mid_planes)
        self.shuffle1 = ShuffleBlock(groups=g)
        self.conv2 = Conv2d(mid_planes, mid_planes, kernel_size=3, stride=stride, padding=1,
                            groups=mid_planes, bias=False)
        self.bn2 = BatchNorm2d(mid_planes)
        self.conv3 = Conv2d(mid_planes, out_planes, kernel_size=1, groups=groups, bias=False)
        self.bn3 = BatchNorm2d(out_planes)
        self.shortcut = Sequential()
        if stride == 2:
            self.shortcut = Sequential(AvgPool2d(3, stride=2, padding=1))

    def forward(self, x):
        out = self.shuffle1(self.bn1(self.conv1(x), act="relu"))
        out = self.bn2(self.conv2(out), act="relu")
        res = self.shortcut(x)
        if self.stride == 2:
            return F.relu(F.cat([self.bn3(self.conv3(out)), res], 1))
        return self.bn3(self.conv3(out), act="relu", residual=res)


class ShuffleNet(tnn.Module):
    def __init__(self, cfg):
        super().__init__()
        out_planes, num_blocks, groups = cfg["out_planes"], cfg["num_blocks"], cfg["groups"]
        self.conv1 = Conv2d(3, 24, kernel_size=1, bias=False)
        self.bn1 = BatchNorm2d(24)
        self.in_planes = 24
        self.layer1 = self._make_layer(out_planes[0], num_blocks[0], groups)
        self.layer2 = self._make_layer(out_planes[1], num_blocks[1], groups)
        self.layer3 = self._make_layer(out_planes[2], num_blocks[2], groups)
        self.linear = Linear(out_planes[2], 10)

    def _make_layer(self, out_planes, num_blocks, groups):
        layers = []
        for i in range(num_blocks):
            stride = 2 if i == 0 else 1
            cat_planes = self.in_planes if i == 0 else 0
            layers.append(Bottleneck(self.in_planes, out_planes - cat_planes, stride=stride, groups=groups))
            self.in_planes = out_planes
        return Sequential(*layers)

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.layer3(self.layer2(self.layer1(out)))
        return F.pool_linear(out, 4, self.linear)


def ShuffleNetG2():
    return ShuffleNet({"out_planes": [200, 400, 800], "num_blocks": [4, 8, 4], "groups": 2})


def ShuffleNetG3():
    return ShuffleNet({"out_planes": [240, 480, 960], "num_blocks": [4, 8, 4], "groups": 3})
