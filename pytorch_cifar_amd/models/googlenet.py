"""GoogLeNet / Inception-v1, CIFAR variant (parity: reference models/googlenet.py:7-98).

Each branch is the same Sequential(Conv2d(bias), BatchNorm2d, ReLU, ...) as the reference, run
by the fused Sequential; the 5x5 branch is two 3x3 convs (googlenet.py:28-38)."""
import torch.nn as tnn

from ..nn import AvgPool2d, BatchNorm2d, Conv2d, Linear, MaxPool2d, ReLU, Sequential
from ..nn import functional as F


def _cbr(cin, cout, k):
    return [Conv2d(cin, cout, kernel_size=k, padding=k // 2), BatchNorm2d(cout), ReLU(True)]


class Inception(tnn.Module):
    def __init__(self, in_planes, n1x1, n3x3red, n3x3, n5x5red, n5x5, pool_planes):
        super().__init__()
        self.b1 = Sequential(*_cbr(in_planes, n1x1, 1))
        self.b2 = Sequential(*_cbr(in_planes, n3x3red, 1), *_cbr(n3x3red, n3x3, 3))
        self.b3 = Sequential(*_cbr(in_planes, n5x5red, 1), *_cbr(n5x5red, n5x5, 3), *_cbr(n5x5, n5x5, 3))
        self.b4 = Sequential(MaxPool2d(3, stride=1, padding=1), *_cbr(in_planes, pool_planes, 1))

    def forward(self, x):
        branches = (self.b1, self.b2, self.b3, self.b4)
        widths = [b[-2].num_features for b in branches]
        if F.ChannelSlab.usable(x, widths):
            # zero-copy concat: each branch's final BN+ReLU writes its channel slice of
            # the output slab; the slab's gradient reaches the branches as strided views
            slab = F.ChannelSlab(x, widths)
            return slab.cat([b(x, out=slab.dest(i)) for i, b in enumerate(branches)])
        return F.cat([b(x) for b in branches], 1)


class GoogLeNet(tnn.Module):
    def __init__(self):
        super().__init__()
        self.pre_layers = Sequential(*_cbr(3, 192, 3))
        self.a3 = Inception(192, 64, 96, 128, 16, 32, 32)
        self.b3 = Inception(256, 128, 128, 192, 32, 96, 64)
        self.maxpool = MaxPool2d(3, stride=2, padding=1)
        self.a4 = Inception(480, 192, 96, 208, 16, 48, 64)
        self.b4 = Inception(512, 160, 112, 224, 24, 64, 64)
        self.c4 = Inception(512, 128, 128, 256, 24, 64, 64)
        self.d4 = Inception(512, 112, 144, 288, 32, 64, 64)
        self.e4 = Inception(528, 256, 160, 320, 32, 128, 128)
        self.a5 = Inception(832, 256, 160, 320, 32, 128, 128)
        self.b5 = Inception(832, 384, 192, 384, 48, 128, 128)
        self.avgpool = AvgPool2d(8, stride=1)
        self.linear = Linear(1024, 10)

    def forward(self, x):
        out = self.b3(self.a3(self.pre_layers(x)))
        out = self.maxpool(out)
        for m in (self.a4, self.b4, self.c4, self.d4, self.e4):
            out = m(out)
        out = self.maxpool(out)
        out = self.b5(self.a5(out))
        # avgpool(8) over the 8x8 map + Linear (googlenet.py:95-98) as the fused head kernel
        return F.pool_linear(out, self.avgpool.kernel_size, self.linear)
