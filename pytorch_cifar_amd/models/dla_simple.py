"""SimpleDLA — main.py's default model (parity: reference models/dla_simple.py:16-116).

Recursive binary aggregation tree; ``Root`` concatenates children and applies 1x1 conv + fused
BN+ReLU. Residual BasicBlocks are the fused ResNet blocks."""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, ReLU, Sequential
from ..nn import functional as F
from ._blocks import shortcut_kwargs


class BasicBlock(tnn.Module):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = Conv2d(in_planes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.conv2 = Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.shortcut = Sequential()
        if stride != 1 or in_planes != self.expansion * planes:
            self.shortcut = Sequential(
                Conv2d(in_planes, self.expansion * planes, kernel_size=1, stride=stride, bias=False),
                BatchNorm2d(self.expansion * planes))

    def forward(self, x, out=None):
        y = self.bn1(self.conv1(x), act="relu")
        return self.bn2(self.conv2(y), act="relu", out=out, **shortcut_kwargs(self.shortcut, x))


class Root(tnn.Module):
    def __init__(self, in_channels, out_channels, kernel_size=1):
        super().__init__()
        self.conv = Conv2d(in_channels, out_channels, kernel_size, stride=1,
                           padding=(kernel_size - 1) // 2, bias=False)
        self.bn = BatchNorm2d(out_channels)

    def forward(self, xs, out=None):
        return self.forward_cat(F.cat(list(xs), 1), out)

    def forward_cat(self, x, out=None):
        return self.bn(self.conv(x), act="relu", out=out)


class Tree(tnn.Module):
    def __init__(self, block, in_channels, out_channels, level=1, stride=1):
        super().__init__()
        self.stride = stride
        self.out_channels = out_channels
        self.root = Root(2 * out_channels, out_channels)
        if level == 1:
            self.left_tree = block(in_channels, out_channels, stride=stride)
            self.right_tree = block(out_channels, out_channels, stride=1)
        else:
            self.left_tree = Tree(block, in_channels, out_channels, level=level - 1, stride=stride)
            self.right_tree = Tree(block, out_channels, out_channels, level=level - 1, stride=1)

    def forward(self, x, out=None):
        C = self.out_channels
        if F.ChannelSlab.usable(x, [C, C]):
            # zero-copy Root concat: both children write their final BN output into their slice
            # of one slab, which the root conv reads whole; the right child gets a dense copy of
            # the left output (one C-wide pass instead of the 2C concat + split)
            hw = ((x.shape[2] - 1) // self.stride + 1, (x.shape[3] - 1) // self.stride + 1)
            slab = F.ChannelSlab(x, [C, C], hw)
            out1 = self.left_tree(x, out=slab.dest(0))
            out2 = self.right_tree(F.dense_copy(out1), out=slab.dest(1))
            return self.root.forward_cat(slab.cat([out1, out2]), out=out)
        out1 = self.left_tree(x)
        out2 = self.right_tree(out1)
        return self.root([out1, out2], out=out)


def _stem(cin, cout):
    return Sequential(Conv2d(cin, cout, kernel_size=3, stride=1, padding=1, bias=False),
                      BatchNorm2d(cout), ReLU(True))


class SimpleDLA(tnn.Module):
    def __init__(self, block=BasicBlock, num_classes=10):
        super().__init__()
        self.base = _stem(3, 16)
        self.layer1 = _stem(16, 16)
        self.layer2 = _stem(16, 32)
        self.layer3 = Tree(block, 32, 64, level=1, stride=1)
        self.layer4 = Tree(block, 64, 128, level=2, stride=2)
        self.layer5 = Tree(block, 128, 256, level=2, stride=2)
        self.layer6 = Tree(block, 256, 512, level=1, stride=2)
        self.linear = Linear(512, num_classes)

    def forward(self, x):
        out = self.layer2(self.layer1(self.base(x)))
        out = self.layer6(self.layer5(self.layer4(self.layer3(out))))
        return F.pool_linear(out, 4, self.linear)
