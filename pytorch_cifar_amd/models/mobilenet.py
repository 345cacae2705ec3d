"""MobileNet v1 (parity: reference models/mobilenet.py:11-52): depthwise 3x3 + pointwise 1x1
blocks, each conv followed by a fused BN+ReLU pass."""
import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F


class Block(tnn.Module):
    """Depthwise conv + pointwise conv"""

    def __init__(self, in_planes, out_planes, stride=1):
        super().__init__()
        self.conv1 = Conv2d(in_planes, in_planes, kernel_size=3, stride=stride, padding=1,
                            groups=in_planes, bias=False)
        self.bn1 = BatchNorm2d(in_planes)
        self.conv2 = Conv2d(in_planes, out_planes, kernel_size=1, stride=1, padding=0, bias=False)
        self.bn2 = BatchNorm2d(out_planes)

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        return self.bn2(self.conv2(out), act="relu")


class MobileNet(tnn.Module):
    # (128, 2): 128 output planes with stride 2; plain ints use stride 1
    cfg = [64, (128, 2), 128, (256, 2), 256, (512, 2), 512, 512, 512, 512, 512, (1024, 2), 1024]

    def __init__(self, num_classes=10):
        super().__init__()
        self.conv1 = Conv2d(3, 32, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = BatchNorm2d(32)
        self.layers = self._make_layers(in_planes=32)
        self.linear = Linear(1024, num_classes)

    def _make_layers(self, in_planes):
        layers = []
        for x in self.cfg:
            out_planes, stride = (x, 1) if isinstance(x, int) else x
            layers.append(Block(in_planes, out_planes, stride))
            in_planes = out_planes
        return Sequential(*layers)

    def forward(self, x):
        out = self.layers(self.bn1(self.conv1(x), act="relu"))
        return F.pool_linear(out, 2, self.linear)
