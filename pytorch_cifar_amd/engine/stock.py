"""Like-for-like comparator: the reference training step on stock PyTorch-ROCm.

What main_dist.py runs per step (SGD 0.9/5e-4, CE, autocast) with the library kernels PyTorch
ships for ROCm (MIOpen convolutions/BN, hipBLASLt linear, RCCL DDP), in the best stock
configuration: NCHW + bf16 autocast (its faster layout on MI355X), synthetic batches already
on the GPU. Used by
``bench.py --baseline`` to put our number next to the stock one measured on the same box.
ResNet-18 is built from torch.nn layers with the CIFAR ResNet topology of models/resnet.py; any
other zoo model runs our model code with every op routed to stock torch (``reference_kernels``).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F


def _cbr(cin, cout, k, s):
    return nn.Sequential(nn.Conv2d(cin, cout, k, s, k // 2, bias=False), nn.BatchNorm2d(cout))


class _Res(nn.Module):
    def __init__(self, cin, cout, s):
        super().__init__()
        self.a = _cbr(cin, cout, 3, s)
        self.b = _cbr(cout, cout, 3, 1)
        self.proj = _cbr(cin, cout, 1, s) if (s != 1 or cin != cout) else None

    def forward(self, x):
        y = self.b(F.relu(self.a(x)))
        return F.relu(y + (self.proj(x) if self.proj is not None else x))


def stock_resnet18(num_classes=10):
    widths, blocks = (64, 128, 256, 512), (2, 2, 2, 2)
    layers, cin = [_cbr(3, 64, 3, 1), nn.ReLU()], 64
    for i, (w, n) in enumerate(zip(widths, blocks)):
        for j in range(n):
            layers.append(_Res(cin, w, 2 if (j == 0 and i > 0) else 1))
            cin = w
    layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(512, num_classes)]
    return nn.Sequential(*layers)


def build_stock_step(model_name, per_rank_batch, device, ctx, images, labels):
    torch.manual_seed(0)
    ref_ctx = None
    if model_name == "ResNet18":
        net = stock_resnet18()
    else:
        # any other zoo model: our model code run entirely through stock torch ops
        # (F.conv2d / F.batch_norm / ... = MIOpen / hipBLASLt), i.e. the reference's op sequence
        from .. import models
        from ..ops.functional import reference_kernels

        net = models.build_model(model_name)
        ref_ctx = reference_kernels
    # layout: NCHW by default — measured on MI355X it is stock's faster layout (ResNet-18 bs1024:
    # 52.6k img/s NCHW vs 43.4k channels_last); PCA_STOCK_NCHW=0 selects channels_last
    nchw = os.environ.get("PCA_STOCK_NCHW", "1") == "1"
    net = net.to(device)
    if not nchw:
        net = net.to(memory_format=torch.channels_last)
    model = net
    if ctx.world > 1:
        model = nn.parallel.DistributedDataParallel(net, device_ids=[device.index])
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4)
    # MIOpen exhaustive find per shape (cudnn.benchmark) takes minutes on the mobile zoo's many
    # depthwise shapes; it is used for ResNet-18 (the reference sets it, main.py:75)
    torch.backends.cudnn.benchmark = model_name == "ResNet18"
    mean = torch.tensor((0.4914, 0.4822, 0.4465), device=device).view(1, 3, 1, 1)
    std = torch.tensor((0.2023, 0.1994, 0.2010), device=device).view(1, 3, 1, 1)
    imgs = torch.from_numpy(images).to(device)
    labs = torch.from_numpy(labels).to(device)
    n = imgs.shape[0]
    state = {"i": 0}

    def run():
        i = state["i"]
        idx = torch.arange(i, i + per_rank_batch, device=device) % n
        state["i"] = (i + per_rank_batch) % n
        x = imgs.index_select(0, idx).permute(0, 3, 1, 2).float().div_(255)
        x = ((x - mean) / std).contiguous(memory_format=torch.contiguous_format if nchw else torch.channels_last)
        y = labs.index_select(0, idx)
        opt.zero_grad(set_to_none=True)
        if ref_ctx is not None:
            with ref_ctx(), torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(x)
                loss = F.cross_entropy(out.float(), y)
            with ref_ctx():
                loss.backward()
        else:
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = model(x)
                loss = F.cross_entropy(out, y)
            loss.backward()
        opt.step()

    return run, {"comparator": "torch.nn + MIOpen + autocast bf16 + " + ("NCHW" if nchw else "channels_last")}
