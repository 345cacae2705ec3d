"""LeNet-5 for CIFAR (parity: reference models/lenet.py:5-23). The BASELINE CPU plumbing config.

On the GPU its 3->6 and 6->16 5x5 convs (channel counts below the MFMA tile) run on the generic
direct-convolution kernels."""
import torch.nn as tnn

from ..nn import Conv2d, Linear
from ..nn import functional as F


class LeNet(tnn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = Conv2d(3, 6, 5)
        self.conv2 = Conv2d(6, 16, 5)
        self.fc1 = Linear(16 * 5 * 5, 120)
        self.fc2 = Linear(120, 84)
        self.fc3 = Linear(84, 10)

    def forward(self, x):
        out = F.max_pool2d(F.relu(self.conv1(x, want_stats=False)), 2)
        out = F.max_pool2d(F.relu(self.conv2(out, want_stats=False)), 2)
        out = out.reshape(out.size(0), -1)
        out = F.relu(self.fc1(out))
        out = F.relu(self.fc2(out))
        return self.fc3(out)
