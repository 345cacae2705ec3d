"""Flat parameter / gradient / momentum arenas (memory laid out for whole-model kernels).

All trainable parameters of a model are re-homed into ONE contiguous fp32 buffer (each parameter
becomes a view with its original shape and strides — conv weights stay channels_last), gradients
into a second one and SGD momentum into a third. Consequences:

* ``zero_grad`` is one memset; native backward kernels accumulate into stable addresses;
* the optimizer step is one multi-tensor launch over three flat arrays;
* the data-parallel engine's all-reduce buckets are contiguous slices of the gradient arena
  (``gradient_as_bucket_view``), laid out in reverse registration order so buckets fill in
  backward order (the DDP Reducer's bucket assignment);
* parameter state broadcast at start-up (C3) is one collective.

``state_dict`` is unaffected: parameters keep their module attributes, names and shapes.
"""
from __future__ import annotations

import torch


def _physical_shape(p: torch.Tensor):
    if p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous():
        n, c, h, w = p.shape
        return (n, h, w, c), (0, 3, 1, 2)
    return tuple(p.shape), None


class ParamArena:
    def __init__(self, params, reverse: bool = True, align: int = 64):
        params = [p for p in params if p.requires_grad]
        seen, uniq = set(), []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        self.params = uniq
        order = list(reversed(uniq)) if reverse else list(uniq)
        self.order = order
        dev = uniq[0].device
        self.offsets = {}
        off = 0
        for p in order:
            self.offsets[id(p)] = (off, p.numel())
            off += (p.numel() + align - 1) // align * align
        self.numel = off
        self.param_flat = torch.zeros(off, dtype=torch.float32, device=dev)
        self.grad_flat = torch.zeros(off, dtype=torch.float32, device=dev)
        self.mom_flat = None
        for p in order:
            pv = self.view(self.param_flat, p)
            pv.copy_(p.detach())
            p.data = pv
            p.grad = self.view(self.grad_flat, p)

    def view(self, flat: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
        off, n = self.offsets[id(p)]
        shape, perm = _physical_shape(p)
        v = flat[off: off + n].view(shape)
        return v.permute(*perm) if perm is not None else v

    def zero_grad(self):
        self.grad_flat.zero_()

    def ensure_momentum(self):
        if self.mom_flat is None:
            self.mom_flat = torch.zeros_like(self.param_flat)
        return self.mom_flat

    def slice_of(self, p):
        off, n = self.offsets[id(p)]
        return off, n


class BufferArena:
    """Flat copies of module buffers (BN running stats) per dtype, for one-shot broadcasts."""

    def __init__(self, module: torch.nn.Module):
        bufs = [b for b in module.buffers() if b is not None]
        self.groups = {}
        for b in bufs:
            self.groups.setdefault(b.dtype, []).append(b)
        self.flats = {}
        for dt, lst in self.groups.items():
            total = sum(b.numel() for b in lst)
            flat = torch.empty(total, dtype=dt, device=lst[0].device)
            off = 0
            for b in lst:
                n = b.numel()
                flat[off: off + n].copy_(b.reshape(-1))
                b.data = flat[off: off + n].view(b.shape)
                off += n
            self.flats[dt] = flat

    def flat_tensors(self):
        return list(self.flats.values())
