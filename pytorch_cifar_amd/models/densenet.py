"""DenseNet121/169/201/161 and densenet_cifar (parity: reference models/densenet.py:9-99).

Pre-activation dense layers (BN-ReLU-1x1 -> BN-ReLU-3x3, concat [new, x]) with BN+ReLU fused;
the BNs read concatenated tensors, so their statistics come from the standalone reduction
kernel rather than a conv epilogue."""
import math

import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F


class Bottleneck(tnn.Module):
    def __init__(self, in_planes, growth_rate):
        super().__init__()
        self.bn1 = BatchNorm2d(in_planes)
        self.conv1 = Conv2d(in_planes, 4 * growth_rate, kernel_size=1, bias=False)
        self.bn2 = BatchNorm2d(4 * growth_rate)
        self.conv2 = Conv2d(4 * growth_rate, growth_rate, kernel_size=3, padding=1, bias=False)

    def forward(self, x, slab=None):
        out = self.conv1(self.bn1(x, act="relu"))
        out = self.conv2(self.bn2(out, act="relu"), want_stats=False)
        if slab is not None:
            return slab.append(out, x)     # zero-copy: x is the slab's suffix, out goes left of it
        return F.cat([out, x], 1)


def dense_block(block, x):
    """Run a dense block's layers; on the GPU the concatenations share one slab (F.DenseSlab)."""
    layers = list(block)
    g = layers[0].conv2.out_channels
    if F.DenseSlab.usable(x, g, len(layers)):
        slab = F.DenseSlab(x, g, len(layers), training=layers[0].bn1.training)
        x = slab.start(x)
        for layer in layers:
            x = layer(x, slab)
        return x
    for layer in layers:
        x = layer(x)
    return x


class Transition(tnn.Module):
    def __init__(self, in_planes, out_planes):
        super().__init__()
        self.bn = BatchNorm2d(in_planes)
        self.conv = Conv2d(in_planes, out_planes, kernel_size=1, bias=False)

    def forward(self, x):
        # avg_pool2d(conv1x1(z), 2) == conv1x1(avg_pool2d(z, 2)) exactly (a bias-free 1x1 conv is
        # a per-pixel linear map, densenet.py:31-32): pooling first runs the conv on a quarter of
        # the pixels (4x fewer FLOPs and conv bytes)
        return self.conv(F.avg_pool2d(self.bn(x, act="relu"), 2), want_stats=False)


class DenseNet(tnn.Module):
    def __init__(self, block, nblocks, growth_rate=12, reduction=0.5, num_classes=10):
        super().__init__()
        self.growth_rate = growth_rate
        planes = 2 * growth_rate
        self.conv1 = Conv2d(3, planes, kernel_size=3, padding=1, bias=False)
        for i in range(4):
            setattr(self, f"dense{i + 1}", self._make_dense_layers(block, planes, nblocks[i]))
            planes += nblocks[i] * growth_rate
            if i < 3:
                out_planes = int(math.floor(planes * reduction))
                setattr(self, f"trans{i + 1}", Transition(planes, out_planes))
                planes = out_planes
        self.bn = BatchNorm2d(planes)
        self.linear = Linear(planes, num_classes)

    def _make_dense_layers(self, block, in_planes, nblock):
        layers = []
        for _ in range(nblock):
            layers.append(block(in_planes, self.growth_rate))
            in_planes += self.growth_rate
        return Sequential(*layers)

    def forward(self, x):
        out = self.conv1(x, want_stats=False)
        out = self.trans1(dense_block(self.dense1, out))
        out = self.trans2(dense_block(self.dense2, out))
        out = self.trans3(dense_block(self.dense3, out))
        out = dense_block(self.dense4, out)
        return F.pool_linear(self.bn(out, act="relu"), 4, self.linear)


def DenseNet121():
    return DenseNet(Bottleneck, [6, 12, 24, 16], growth_rate=32)


def DenseNet169():
    return DenseNet(Bottleneck, [6, 12, 32, 32], growth_rate=32)


def DenseNet201():
    return DenseNet(Bottleneck, [6, 12, 48, 32], growth_rate=32)


def DenseNet161():
    return DenseNet(Bottleneck, [6, 12, 36, 24], growth_rate=48)


def densenet_cifar():
    return DenseNet(Bottleneck, [6, 12, 24, 16], growth_rate=12)
