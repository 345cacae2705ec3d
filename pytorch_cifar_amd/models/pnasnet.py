"""PNASNet-A / PNASNet-B (parity: reference models/pnasnet.py:10-116).

``SepConv`` is the reference's depthwise-only conv (groups=in_planes, channel multiplier 2 in the
stride-2 cells, k in {3, 5, 7}) + BN. The two-branch joins ``relu(a + b)`` of the cells fuse
both BatchNorms, the add and the ReLU into one pass (``residual_bn``)."""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F


class SepConv(tnn.Module):
    """Separable Convolution."""

    def __init__(self, in_planes, out_planes, kernel_size, stride):
        super().__init__()
        self.conv1 = Conv2d(in_planes, out_planes, kernel_size, stride, padding=(kernel_size - 1) // 2,
                            bias=False, groups=in_planes)
        self.bn1 = BatchNorm2d(out_planes)

    def forward(self, x):
        return self.bn1(self.conv1(x))


def _join_relu(a: SepConv, xa, b_bn, b_pre):
    """relu(a.bn1(a.conv1(xa)) + b_bn(b_pre)) in one fused BN/residual/ReLU pass."""
    return a.bn1(a.conv1(xa), act="relu", residual_bn=(b_bn, b_pre))


class CellA(tnn.Module):
    def __init__(self, in_planes, out_planes, stride=1):
        super().__init__()
        self.stride = stride
        self.sep_conv1 = SepConv(in_planes, out_planes, kernel_size=7, stride=stride)
        if stride == 2:
            self.conv1 = Conv2d(in_planes, out_planes, kernel_size=1, stride=1, padding=0, bias=False)
            self.bn1 = BatchNorm2d(out_planes)

    def forward(self, x):
        y2 = F.max_pool2d(x, kernel_size=3, stride=self.stride, padding=1)
        if self.stride == 2:
            return _join_relu(self.sep_conv1, x, self.bn1, self.conv1(y2))
        return self.sep_conv1.bn1(self.sep_conv1.conv1(x), act="relu", residual=y2)


class CellB(tnn.Module):
    def __init__(self, in_planes, out_planes, stride=1):
        super().__init__()
        self.stride = stride
        self.sep_conv1 = SepConv(in_planes, out_planes, kernel_size=7, stride=stride)
        self.sep_conv2 = SepConv(in_planes, out_planes, kernel_size=3, stride=stride)
        self.sep_conv3 = SepConv(in_planes, out_planes, kernel_size=5, stride=stride)
        if stride == 2:
            self.conv1 = Conv2d(in_planes, out_planes, kernel_size=1, stride=1, padding=0, bias=False)
            self.bn1 = BatchNorm2d(out_planes)
        self.conv2 = Conv2d(2 * out_planes, out_planes, kernel_size=1, stride=1, padding=0, bias=False)
        self.bn2 = BatchNorm2d(out_planes)

    def forward(self, x):
        b1 = _join_relu(self.sep_conv1, x, self.sep_conv2.bn1, self.sep_conv2.conv1(x))
        y3 = F.max_pool2d(x, kernel_size=3, stride=self.stride, padding=1)
        if self.stride == 2:
            b2 = _join_relu(self.sep_conv3, x, self.bn1, self.conv1(y3))
        else:
            b2 = self.sep_conv3.bn1(self.sep_conv3.conv1(x), act="relu", residual=y3)
        return self.bn2(self.conv2(F.cat([b1, b2], 1)), act="relu")


class PNASNet(tnn.Module):
    def __init__(self, cell_type, num_cells, num_planes):
        super().__init__()
        self.in_planes = num_planes
        self.cell_type = cell_type
        self.conv1 = Conv2d(3, num_planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = BatchNorm2d(num_planes)
        self.layer1 = self._make_layer(num_planes, num_cells=6)
        self.layer2 = self._downsample(num_planes * 2)
        self.layer3 = self._make_layer(num_planes * 2, num_cells=6)
        self.layer4 = self._downsample(num_planes * 4)
        self.layer5 = self._make_layer(num_planes * 4, num_cells=6)
        self.linear = Linear(num_planes * 4, 10)

    def _make_layer(self, planes, num_cells):
        layers = []
        for _ in range(num_cells):
            layers.append(self.cell_type(self.in_planes, planes, stride=1))
            self.in_planes = planes
        return Sequential(*layers)

    def _downsample(self, planes):
        layer = self.cell_type(self.in_planes, planes, stride=2)
        self.in_planes = planes
        return layer

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        for m in (self.layer1, self.layer2, self.layer3, self.layer4, self.layer5):
            out = m(out)
        return F.pool_linear(out, 8, self.linear)


def PNASNetA():
    return PNASNet(CellA, num_cells=6, num_planes=44)


def PNASNetB():
    return PNASNet(CellB, num_cells=6, num_planes=32)
