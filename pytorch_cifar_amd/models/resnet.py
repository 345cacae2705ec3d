"""ResNet18/34/50/101/152 for CIFAR-10 (parity: reference models/resnet.py:16-160).

Same constructor names/signatures (including the ``amp`` flag of this fork), module names and
state_dict keys. Each residual block tail ``relu(bn2(conv2(out)) + shortcut(x))`` is a single fused
BatchNorm/residual/ReLU pass; with a projection shortcut both BatchNorms are folded into it.
``amp`` is accepted for API parity: on MI355X the compute dtype is always bf16 (no loss scaling).
"""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F
from ._blocks import shortcut_kwargs


class BasicBlock(tnn.Module):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1, amp=False):
        super().__init__()
        self.amp = amp
        self.conv1 = Conv2d(in_planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.shortcut = Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = Sequential(
                Conv2d(in_planes, self.expansion * planes, kernel_size=1, stride=stride, bias=False),
                BatchNorm2d(self.expansion * planes),
            )

    def forward(self, x):
        # conv2(relu(bn1(conv1(x)))): on the layer-1 geometry conv2 applies bn1 + ReLU on its own
        # loads (F.bn_act_conv; elsewhere the plain composition)
        out = F.bn_act_conv(self.bn1, self.conv1(x), "relu", self.conv2)
        return self.bn2(out, act="relu", **shortcut_kwargs(self.shortcut, x))


class Bottleneck(tnn.Module):
    expansion = 4

    def __init__(self, in_planes, planes, stride=1, amp=False):
        super().__init__()
        self.amp = amp
        self.conv1 = Conv2d(in_planes, planes, kernel_size=1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.conv3 = Conv2d(planes, self.expansion * planes, kernel_size=1, bias=False)
        self.bn3 = BatchNorm2d(self.expansion * planes)
        self.shortcut = Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = Sequential(
                Conv2d(in_planes, self.expansion * planes, kernel_size=1, stride=stride, bias=False),
                BatchNorm2d(self.expansion * planes),
            )

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.bn2(self.conv2(out), act="relu")
        return self.bn3(self.conv3(out), act="relu", **shortcut_kwargs(self.shortcut, x))


class ResNet(tnn.Module):
    def __init__(self, block, num_blocks, num_classes=10, amp=False):
        super().__init__()
        self.in_planes = 64
        self.amp = amp
        self.conv1 = Conv2d(3, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, num_blocks[0], stride=1)
        self.layer2 = self._make_layer(block, 128, num_blocks[1], stride=2)
        self.layer3 = self._make_layer(block, 256, num_blocks[2], stride=2)
        self.layer4 = self._make_layer(block, 512, num_blocks[3], stride=2)
        self.linear = Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, num_blocks, stride):
        layers = []
        for s in [stride] + [1] * (num_blocks - 1):
            layers.append(block(self.in_planes, planes, s, amp=self.amp))
            self.in_planes = planes * block.expansion
        return Sequential(*layers)

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.layer1(out)
        out = self.layer2(out)
        out = self.layer3(out)
        out = self.layer4(out)
        return F.pool_linear(out, 4, self.linear)


def ResNet18(amp=False):
    return ResNet(BasicBlock, [2, 2, 2, 2], amp=amp)


def ResNet34(amp=False):
    return ResNet(BasicBlock, [3, 4, 6, 3], amp=amp)


def ResNet50(amp=False):
    return ResNet(Bottleneck, [3, 4, 6, 3], amp=amp)


def ResNet101(amp=False):
    return ResNet(Bottleneck, [3, 4, 23, 3], amp=amp)


def ResNet152(amp=False):
    return ResNet(Bottleneck, [3, 8, 36, 3], amp=amp)
