"""VGG11/13/16/19 (parity: reference models/vgg.py:6-38).

``features`` is the same flat Sequential (Conv2d(bias) / BatchNorm2d / ReLU triples, MaxPool2d,
trailing AvgPool2d(1, 1)) so state_dict keys match (``features.0.weight`` ...); the fused
Sequential runs each BatchNorm2d+ReLU pair as one pass and the conv epilogue feeds it statistics.
"""
import torch.nn as tnn

from ..nn import AvgPool2d, BatchNorm2d, Conv2d, Linear, MaxPool2d, ReLU, Sequential
from ..nn import functional as F

cfg = {
    "VGG11": [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG13": [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    "VGG16": [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
    "VGG19": [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M",
              512, 512, 512, 512, "M"],
}


class VGG(tnn.Module):
    def __init__(self, vgg_name):
        super().__init__()
        self.features = self._make_layers(cfg[vgg_name])
        self.classifier = Linear(512, 10)

    @staticmethod
    def _make_layers(spec):
        layers, c = [], 3
        for v in spec:
            if v == "M":
                layers.append(MaxPool2d(kernel_size=2, stride=2))
            else:
                layers += [Conv2d(c, v, kernel_size=3, padding=1), BatchNorm2d(v), ReLU(inplace=True)]
                c = v
        layers.append(AvgPool2d(kernel_size=1, stride=1))
        return Sequential(*layers)

    def forward(self, x):
        out = self.features(x)
        # flatten of the 1x1 map + Linear (vgg.py:21-23) as the fused head kernel
        return F.pool_linear(out, 1, self.classifier)
