"""Single-process data parallelism for ``main.py`` (parity: main.py:73-74 ``nn.DataParallel``).

* One visible GPU (the common MI355X case): a thin wrapper whose only job is API/checkpoint
  parity — the model lives in ``.module`` so ``state_dict`` keys carry the reference's
  ``module.`` prefix — and the forward runs directly (no replicate/scatter/gather per step).
* Several GPUs in one process: the replicate / scatter / parallel_apply / gather schedule of
  ``torch.nn.DataParallel``, which works unchanged with the native ops
  because their backward returns gradients of non-leaf (replicated) parameters through autograd.
  For multi-GPU throughput use ``main_dist.py`` (one process per GPU, RCCL buckets).
"""
from __future__ import annotations

import torch
import torch.nn as nn


class DataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids=None, output_device=None):
        super().__init__()
        self.module = module
        if device_ids is None:
            device_ids = list(range(torch.cuda.device_count())) if torch.cuda.is_available() else []
        self.device_ids = device_ids
        self._torch_dp = None
        if len(device_ids) > 1:
            self._torch_dp = nn.DataParallel(module, device_ids=device_ids, output_device=output_device)

    def forward(self, *inputs, **kwargs):
        if self._torch_dp is not None:
            return self._torch_dp(*inputs, **kwargs)
        return self.module(*inputs, **kwargs)
