#!/usr/bin/env python3
"""Localise a production-step mismatch: run the production test's two steps (ResNet-18 by default)
on the native path and the fp32 stock oracle, with forward hooks on every module, and print the
relative error of each module output on the compared (second) step, plus logits / gradients.

  python tools/diag/prod_layers.py --batch 1024 [--model ResNet18] [--steps 2]
"""
import argparse
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--model", default="ResNet18")
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.engine.arena import ParamArena
    from pytorch_cifar_amd.ops.functional import (cross_entropy, enable_batched_weight_prep,
                                                  reference_kernels)

    torch.manual_seed(0)
    base = models.MODEL_REGISTRY[a.model]()
    ref = copy.deepcopy(base).cuda().to(memory_format=torch.channels_last)
    nat = copy.deepcopy(base).cuda()
    arena = ParamArena(nat.parameters())
    enable_batched_weight_prep(nat)
    ref.train()
    nat.train()
    outs = {"ref": {}, "nat": {}}

    def hook(tag, name):
        def f(m, i, o):
            if isinstance(o, torch.Tensor):
                outs[tag][name] = o.detach().float().clone()
        return f

    for tag, m in (("ref", ref), ("nat", nat)):
        for n, mod in m.named_modules():
            if n:
                mod.register_forward_hook(hook(tag, n))
    g = torch.Generator(device="cpu").manual_seed(1)
    for it in range(a.steps):
        x = torch.randn(a.batch, 3, 32, 32, generator=g).cuda()
        y = torch.randint(0, 10, (a.batch,), generator=g).cuda()
        for p in ref.parameters():
            p.grad = None
        arena.zero_grad()
        outs["ref"].clear()
        outs["nat"].clear()
        with reference_kernels():
            o_r = ref(x.contiguous(memory_format=torch.channels_last))
            cross_entropy(o_r.float(), y).backward()
        o_n = nat(x)
        cross_entropy(o_n, y).backward()
        torch.cuda.synchronize()
        print(f"step {it}: logits rel {rel(o_n, o_r):.4f}", flush=True)
        for n in outs["ref"]:
            if n in outs["nat"] and outs["nat"][n].shape == outs["ref"][n].shape:
                print(f"  {n:32s} {rel(outs['nat'][n], outs['ref'][n]):.4f}")
        gr = dict(ref.named_parameters())
        worst = sorted(((rel(p.grad, gr[n].grad), n) for n, p in nat.named_parameters()
                        if p.grad is not None and gr[n].grad is not None), reverse=True)[:8]
        print("  worst grads:", [(n, round(e, 4)) for e, n in worst])
        bufs = dict(ref.named_buffers())
        bw = sorted(((rel(b, bufs[n]), n) for n, b in nat.named_buffers() if b.dtype.is_floating_point),
                    reverse=True)[:5]
        print("  worst buffers:", [(n, round(e, 4)) for e, n in bw], flush=True)


if __name__ == "__main__":
    main()
