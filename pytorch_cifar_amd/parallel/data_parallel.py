"""Single-device module wrapper with ``nn.DataParallel``'s checkpoint layout (main.py:73-74).

Multi-GPU data parallelism in this framework is one process per GPU on the native RCCL bucket
engine (:mod:`.ddp`): ``main.py`` and the non-``--dist`` path of ``main_dist.py`` — the
reference's ``nn.DataParallel`` workloads (main.py:74, main_dist.py:145-147) —
start one rank per visible GPU themselves (:func:`.launcher.spawn_local_ranks`) and split the
batch across them the way DataParallel's scatter did. Each rank's model lives in ``.module``, so
checkpoints keep the reference's ``module.`` keys either way.

This wrapper covers the remaining single-process case: the model on one device, forward called
directly (no replicate / scatter / gather per step), ``module.`` prefixed ``state_dict``. Asking it
for several devices in one process raises and points at the rank-per-GPU launch instead of
silently falling back to stock single-process replication (broadcast_coalesced / reduce_add every
step, no hipGraph, no native buckets).
"""
from __future__ import annotations

import torch.nn as nn


class DataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None):
        super().__init__()
        self.module = module
        if device_ids is None:
            p = next(module.parameters(), None)
            device_ids = [p.device.index] if p is not None and p.device.type == "cuda" else []
        if len(device_ids) > 1:
            raise ValueError(
                "pytorch_cifar_amd.DataParallel is single-device; for several GPUs run one rank per GPU "
                "(main.py / main_dist.py do this by default, or parallel.launcher.spawn_local_ranks) "
                "with parallel.ddp.DistributedDataParallel")
        self.device_ids = device_ids
        self.output_device = output_device

    def forward(self, *inputs, **kwargs):
        return self.module(*inputs, **kwargs)
