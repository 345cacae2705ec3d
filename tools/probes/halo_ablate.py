"""Halo wgrad bottleneck probe (run under rocprofv3 --kernel-trace --stats, one process per
PCA_HALO_ABLATE value: 0 full kernel, 1 no DMA, 2 no MFMA phase, 3 neither): the ResNet-18 3x3
stride-1 weight gradients at the bs128 shard with the configs the step's autotuner picks."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from pytorch_cifar_amd import _native  # noqa: E402

C = _native.lib()
N = int(os.environ.get("PROBE_BATCH", "128"))
shapes = [(64, 32, 35), (128, 16, 35), (256, 8, 35), (512, 4, 34)]   # (C, H, halo cfg)
for ch, h, cfg in shapes:
    x = torch.randn(N, h, h, ch, device="cuda").to(torch.bfloat16)
    dy = torch.randn(N, h, h, ch, device="cuda").to(torch.bfloat16)
    C.conv_trial(1, cfg, -1)
    for _ in range(20):
        C.conv_wgrad(x, dy, 3, 3, 1, 1, 1, None)
    torch.cuda.synchronize()
C.conv_trial(1, -1, -1)
print("done", os.environ.get("PCA_HALO_ABLATE", "0"))
