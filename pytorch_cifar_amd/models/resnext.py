"""ResNeXt29 {2x64d, 4x64d, 8x64d, 32x4d} (parity: reference models/resnext.py:10-87).

Three stages (the reference's layer4 is commented out), 1x1 stem, bottleneck width doubling per
stage. Grouped 3x3 convs with >= 8 channels per group run on the MFMA kernel (one GEMM per
group along grid.z); 32x4d's 4-channel groups use the direct kernel."""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F
from ._blocks import shortcut_kwargs


class Block(tnn.Module):
    expansion = 2

    def __init__(self, in_planes, cardinality=32, bottleneck_width=4, stride=1):
        super().__init__()
        gw = cardinality * bottleneck_width
        self.conv1 = Conv2d(in_planes, gw, kernel_size=1, bias=False)
        self.bn1 = BatchNorm2d(gw)
        self.conv2 = Conv2d(gw, gw, kernel_size=3, stride=stride, padding=1, groups=cardinality, bias=False)
        self.bn2 = BatchNorm2d(gw)
        self.conv3 = Conv2d(gw, self.expansion * gw, kernel_size=1, bias=False)
        self.bn3 = BatchNorm2d(self.expansion * gw)
        self.shortcut = Sequential()
        if stride != 1 or in_planes != self.expansion * gw:
            self.shortcut = Sequential(
                Conv2d(in_planes, self.expansion * gw, kernel_size=1, stride=stride, bias=False),
                BatchNorm2d(self.expansion * gw))

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.bn2(self.conv2(out), act="relu")
        return self.bn3(self.conv3(out), act="relu", **shortcut_kwargs(self.shortcut, x))


class ResNeXt(tnn.Module):
    def __init__(self, num_blocks, cardinality, bottleneck_width, num_classes=10):
        super().__init__()
        self.cardinality = cardinality
        self.bottleneck_width = bottleneck_width
        self.in_planes = 64
        self.conv1 = Conv2d(3, 64, kernel_size=1, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.layer1 = self._make_layer(num_blocks[0], 1)
        self.layer2 = self._make_layer(num_blocks[1], 2)
        self.layer3 = self._make_layer(num_blocks[2], 2)
        self.linear = Linear(cardinality * bottleneck_width * 8, num_classes)

    def _make_layer(self, num_blocks, stride):
        layers = []
        for s in [stride] + [1] * (num_blocks - 1):
            layers.append(Block(self.in_planes, self.cardinality, self.bottleneck_width, s))
            self.in_planes = Block.expansion * self.cardinality * self.bottleneck_width
        self.bottleneck_width *= 2
        return Sequential(*layers)

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.layer3(self.layer2(self.layer1(out)))
        return F.pool_linear(out, 8, self.linear)


def ResNeXt29_2x64d():
    return ResNeXt(num_blocks=[3, 3, 3], cardinality=2, bottleneck_width=64)


def ResNeXt29_4x64d():
    return ResNeXt(num_blocks=[3, 3, 3], cardinality=4, bottleneck_width=64)


def ResNeXt29_8x64d():
    return ResNeXt(num_blocks=[3, 3, 3], cardinality=8, bottleneck_width=64)


def ResNeXt29_32x4d():
    return ResNeXt(num_blocks=[3, 3, 3], cardinality=32, bottleneck_width=4)
