"""ShuffleNetV2(net_size in {0.5, 1, 1.5, 2}) (parity: reference models/shufflenetv2.py:10-152).

Channel split -> (1x1 + BN + ReLU -> depthwise 3x3 + BN -> 1x1 + BN + ReLU) -> concat -> shuffle;
two-branch stride-2 DownBlock. Odd widths (58/116/232 for net_size 1) fall back to the generic
direct-conv and scalar depthwise kernels where the MFMA tile needs multiples of 8.

Inside a stage the blocks hand each other the two SplitBlock halves instead of the joined
tensor: every join but the stage's last is F.cat_shuffle2_split (one interleave pass writing
both halves), so no split / concat pass runs between blocks (K22). At odd widths the second
half is written zero-padded to a multiple of 8 channels, the layout the next block's 1x1 conv
reads in place. Calling a block on its own keeps the reference contract (joined tensor in,
joined tensor out)."""
import os

import torch.nn as tnn

from ..nn import BatchNorm2d, Conv2d, Linear, Sequential
from ..nn import functional as F


def _pad8(c):
    """Width the next block's branch input is held at (zero-padded to a multiple of 8 when its
    odd-width 1x1 conv would otherwise pad it in a pass of its own), 0 = dense."""
    return (c + 7) // 8 * 8 if c % 8 else 0


class ShuffleBlock(tnn.Module):
    def __init__(self, groups=2):
        super().__init__()
        self.groups = groups

    def forward(self, x):
        return F.channel_shuffle(x, self.groups)


class SplitBlock(tnn.Module):
    def __init__(self, ratio):
        super().__init__()
        self.ratio = ratio

    def forward(self, x):
        c = int(x.size(1) * self.ratio)
        return F.split_channels(x, c)


class BasicBlock(tnn.Module):
    def __init__(self, in_channels, split_ratio=0.5):
        super().__init__()
        self.split = SplitBlock(split_ratio)
        c = int(in_channels * split_ratio)
        self.conv1 = Conv2d(c, c, kernel_size=1, bias=False)
        self.bn1 = BatchNorm2d(c)
        self.conv2 = Conv2d(c, c, kernel_size=3, stride=1, padding=1, groups=c, bias=False)
        self.bn2 = BatchNorm2d(c)
        self.conv3 = Conv2d(c, c, kernel_size=1, bias=False)
        self.bn3 = BatchNorm2d(c)
        self.shuffle = ShuffleBlock()

    def forward(self, x):
        x1, x2 = self.split(x)
        return self._join(x1, self._branch(x2))

    def _branch(self, x2):
        out = self.bn2(F.bn_act_dwconv(self.bn1, self.conv1(x2), "relu", self.conv2))
        return self.bn3(self.conv3(out), act="relu")

    def forward_halves(self, x1, x2, split_out=True):
        """forward() on the SplitBlock halves; split_out: return the halves of the result."""
        out = self._branch(x2)
        if split_out and self.shuffle.groups == 2:
            return F.cat_shuffle2_split(x1, out, _pad8(out.shape[1]))
        return self._join(x1, out)

    def _join(self, a, b):
        if self.shuffle.groups == 2 and a.shape == b.shape:
            return F.cat_shuffle2(a, b)          # == shuffle(cat([a, b])), one native pass
        return self.shuffle(F.cat([a, b], 1))


class DownBlock(tnn.Module):
    def __init__(self, in_channels, out_channels):
        super().__init__()
        mid = out_channels // 2
        self.conv1 = Conv2d(in_channels, in_channels, kernel_size=3, stride=2, padding=1,
                            groups=in_channels, bias=False)
        self.bn1 = BatchNorm2d(in_channels)
        self.conv2 = Conv2d(in_channels, mid, kernel_size=1, bias=False)
        self.bn2 = BatchNorm2d(mid)
        self.conv3 = Conv2d(in_channels, mid, kernel_size=1, bias=False)
        self.bn3 = BatchNorm2d(mid)
        self.conv4 = Conv2d(mid, mid, kernel_size=3, stride=2, padding=1, groups=mid, bias=False)
        self.bn4 = BatchNorm2d(mid)
        self.conv5 = Conv2d(mid, mid, kernel_size=1, bias=False)
        self.bn5 = BatchNorm2d(mid)
        self.shuffle = ShuffleBlock()

    def _branches(self, x):
        # the right branch first: its 1x1 conv3 becomes the owner of x's gradient slot, so the
        # left branch's depthwise dgrad (whose backward then runs first) hands its dX to conv3's
        # dgrad epilogue instead of an autograd add (same values either order)
        right = self.bn4(F.bn_act_dwconv(self.bn3, self.conv3(x), "relu", self.conv4))
        left = self.bn2(self.conv2(self.bn1(self.conv1(x))), act="relu")
        return left, self.bn5(self.conv5(right), act="relu")

    def forward(self, x):
        left, right = self._branches(x)
        if self.shuffle.groups == 2 and left.shape == right.shape:
            return F.cat_shuffle2(left, right)
        return self.shuffle(F.cat([left, right], 1))

    def forward_halves(self, x):
        """forward() returned as the next block's SplitBlock halves."""
        left, right = self._branches(x)
        return F.cat_shuffle2_split(left, right, _pad8(left.shape[1]))


class _Stage(Sequential):
    """_make_layer's Sequential (same state_dict keys) running its blocks on SplitBlock halves
    (module docstring); falls back to block-by-block calls when a block carries hooks or a
    split other than the reference's 0.5 / groups 2 / equal-width join."""

    def _halves_ok(self):
        if os.environ.get("PCA_ZERO_COPY_CAT", "1") == "0":
            return False
        blocks = list(self)
        if len(blocks) < 2 or not isinstance(blocks[0], DownBlock):
            return False
        for b in blocks:
            if b._forward_hooks or b._forward_pre_hooks or b.shuffle.groups != 2:
                return False
            if isinstance(b, BasicBlock) and b.split.ratio != 0.5:
                return False
        mid = blocks[0].conv2.out_channels
        return all(b.conv1.in_channels == mid for b in blocks[1:])

    def forward(self, x):
        if not self._halves_ok():
            return super().forward(x)
        blocks = list(self)
        h = blocks[0].forward_halves(x)
        for i, b in enumerate(blocks[1:], 1):
            h = b.forward_halves(*h, split_out=i < len(blocks) - 1)
        return h


class ShuffleNetV2(tnn.Module):
    def __init__(self, net_size):
        super().__init__()
        out_channels = configs[net_size]["out_channels"]
        num_blocks = configs[net_size]["num_blocks"]
        self.conv1 = Conv2d(3, 24, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn1 = BatchNorm2d(24)
        self.in_channels = 24
        self.layer1 = self._make_layer(out_channels[0], num_blocks[0])
        self.layer2 = self._make_layer(out_channels[1], num_blocks[1])
        self.layer3 = self._make_layer(out_channels[2], num_blocks[2])
        self.conv2 = Conv2d(out_channels[2], out_channels[3], kernel_size=1, stride=1, padding=0, bias=False)
        self.bn2 = BatchNorm2d(out_channels[3])
        self.linear = Linear(out_channels[3], 10)

    def _make_layer(self, out_channels, num_blocks):
        layers = [DownBlock(self.in_channels, out_channels)]
        for _ in range(num_blocks):
            layers.append(BasicBlock(out_channels))
            self.in_channels = out_channels
        return _Stage(*layers)

    def forward(self, x):
        out = self.bn1(self.conv1(x), act="relu")
        out = self.layer3(self.layer2(self.layer1(out)))
        out = self.bn2(self.conv2(out), act="relu")
        return F.pool_linear(out, 4, self.linear)


configs = {
    0.5: {"out_channels": (48, 96, 192, 1024), "num_blocks": (3, 7, 3)},
    1: {"out_channels": (116, 232, 464, 1024), "num_blocks": (3, 7, 3)},
    1.5: {"out_channels": (176, 352, 704, 1024), "num_blocks": (3, 7, 3)},
    2: {"out_channels": (224, 488, 976, 2048), "num_blocks": (3, 7, 3)},
}
