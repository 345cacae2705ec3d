#!/usr/bin/env python3
"""Native bf16 step vs the CPU fp32 reference path on a random projection of the logits: logits
error, worst and median per-parameter gradient errors (GPU). Shows which nets have numerically
zero gradients at init (ShuffleNetV2's stacked no-activation BatchNorms: median ~0.93 vs ResNet-18's
~0.30 at batch 8), i.e. where only a relative-to-stock-bf16 comparison is meaningful."""
import copy, sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
import torch
from pytorch_cifar_amd import models
def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()
for name, B in (("ShuffleNetV2_1", 8), ("ShuffleNetV2_1", 32), ("ResNet18", 8)):
    torch.manual_seed(0)
    ref = models.MODEL_REGISTRY[name]()
    nat = copy.deepcopy(ref).cuda()
    x = torch.randn(B, 3, 32, 32)
    dl = torch.randn(B, 10)
    o_r = ref(x); (o_r * dl).sum().backward()
    o_n = nat(x.cuda().contiguous(memory_format=torch.channels_last)); (o_n.float() * dl.cuda()).sum().backward()
    torch.cuda.synchronize()
    gr = dict(ref.named_parameters()); gn = dict(nat.named_parameters())
    errs = sorted(((rel(gn[n].grad, p.grad), n) for n, p in gr.items() if p.grad is not None), reverse=True)
    print(name, B, "logits", round(rel(o_n, o_r), 4), "worst grads", [(round(e, 3), n) for e, n in errs[:4]],
          "median", round(errs[len(errs) // 2][0], 4), flush=True)
