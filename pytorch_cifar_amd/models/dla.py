"""DLA, paper-style tree (parity: reference models/dla.py:11-123).

``level_i`` subtrees are registered with the same dynamic names (``level_1`` ...) and order as
the reference, so state_dict keys match; ``prev_root`` feeds the level>1 aggregation node."""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, ReLU, Sequential
from ..nn import functional as F
from .dla_simple import BasicBlock, Root


class Tree(tnn.Module):
    def __init__(self, block, in_channels, out_channels, level=1, stride=1):
        super().__init__()
        self.level = level
        self.stride = stride
        self.out_channels = out_channels
        if level == 1:
            self.root = Root(2 * out_channels, out_channels)
            self.left_node = block(in_channels, out_channels, stride=stride)
            self.right_node = block(out_channels, out_channels, stride=1)
        else:
            self.root = Root((level + 2) * out_channels, out_channels)
            for i in reversed(range(1, level)):
                setattr(self, "level_%d" % i, Tree(block, in_channels, out_channels, level=i, stride=stride))
            self.prev_root = block(in_channels, out_channels, stride=stride)
            self.left_node = block(out_channels, out_channels, stride=1)
            self.right_node = block(out_channels, out_channels, stride=1)

    def forward(self, x, out=None):
        C = self.out_channels
        n = self.level + 2 if self.level > 1 else 2
        if F.ChannelSlab.usable(x, [C] * n):
            return self._forward_slab(x, C, n, out)
        xs = [self.prev_root(x)] if self.level > 1 else []
        for i in reversed(range(1, self.level)):
            x = getattr(self, "level_%d" % i)(x)
            xs.append(x)
        x = self.left_node(x)
        xs.append(x)
        x = self.right_node(x)
        xs.append(x)
        return self.root(xs, out=out)

    def _forward_slab(self, x, C, n, out):
        """Zero-copy Root concat: every child writes its final BN output into its slice of one
        slab that the root conv reads whole; a child that also feeds the next one hands it a dense
        copy (one C-wide pass instead of the n*C concat + split)."""
        hw = ((x.shape[2] - 1) // self.stride + 1, (x.shape[3] - 1) // self.stride + 1)
        slab = F.ChannelSlab(x, [C] * n, hw)
        parts = []
        if self.level > 1:
            parts.append(self.prev_root(x, out=slab.dest(0)))
        for i in reversed(range(1, self.level)):
            y = getattr(self, "level_%d" % i)(x, out=slab.dest(len(parts)))
            parts.append(y)
            x = F.dense_copy(y)
        y = self.left_node(x, out=slab.dest(len(parts)))
        parts.append(y)
        parts.append(self.right_node(F.dense_copy(y), out=slab.dest(len(parts))))
        return self.root.forward_cat(slab.cat(parts), out=out)


def _stem(cin, cout):
    return Sequential(Conv2d(cin, cout, kernel_size=3, stride=1, padding=1, bias=False),
                      BatchNorm2d(cout), ReLU(True))


class DLA(tnn.Module):
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
