"""SENet18 (parity: reference models/senet.py:10-113): pre-activation blocks with
squeeze-excitation (reduction 16) applied before the residual add. ``BasicBlock`` (the
post-activation variant the reference defines but SENet18 does not use) is kept for API parity."""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F
from ._blocks import shortcut_kwargs


class BasicBlock(tnn.Module):
    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = Conv2d(in_planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.shortcut = Sequential()
        if stride != 1 or in_planes != planes:
            self.shortcut = Sequential(
                Conv2d(in_planes, planes, kernel_size=1, stride=stride, bias=False), BatchNorm2d(planes))
        self.fc1 = Conv2d(planes, planes // 16, kernel_size=1)
        self.fc2 = Conv2d(planes // 16, planes, kernel_size=1)

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = F.se_gate(self.bn2(self.conv2(out)), self.fc1, self.fc2, act="relu")
        kw = shortcut_kwargs(self.shortcut, x)
        sc = kw["residual"] if "residual" in kw else kw["residual_bn"][0](kw["residual_bn"][1])
        return F.add_act(out, sc, "relu")


class PreActBlock(tnn.Module):
    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.bn1 = BatchNorm2d(in_planes)
        self.conv1 = Conv2d(in_planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        if stride != 1 or in_planes != planes:
            self.shortcut = Sequential(Conv2d(in_planes, planes, kernel_size=1, stride=stride, bias=False))
        self.fc1 = Conv2d(planes, planes // 16, kernel_size=1)
        self.fc2 = Conv2d(planes // 16, planes, kernel_size=1)

    def forward(self, x):
        a = self.bn1(x, act="relu")
        sc = self.shortcut(a) if hasattr(self, "shortcut") else x
        out = self.conv2(self.bn2(self.conv1(a), act="relu"), want_stats=False)
        out = F.se_gate(out, self.fc1, self.fc2, act="relu")
        return F.add_act(out, sc)


class SENet(tnn.Module):
    def __init__(self, block, num_blocks, num_classes=10):
        super().__init__()
        self.in_planes = 64
        self.conv1 = Conv2d(3, 64, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, num_blocks[0], stride=1)
        self.layer2 = self._make_layer(block, 128, num_blocks[1], stride=2)
        self.layer3 = self._make_layer(block, 256, num_blocks[2], stride=2)
        self.layer4 = self._make_layer(block, 512, num_blocks[3], stride=2)
        self.linear = Linear(512, num_classes)

    def _make_layer(self, block, planes, num_blocks, stride):
        layers = []
        for s in [stride] + [1] * (num_blocks - 1):
            layers.append(block(self.in_planes, planes, s))
            self.in_planes = planes
        return Sequential(*layers)

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.layer4(self.layer3(self.layer2(self.layer1(out))))
        return F.pool_linear(out, 4, self.linear)


def SENet18():
    return SENet(PreActBlock, [2, 2, 2, 2])
