"""Per-parameter gradient differences of ResNet-18 with / without the dual-BN fused reduce."""
import copy
import sys

import torch

from pytorch_cifar_amd import models
from pytorch_cifar_amd.ops import functional as PF


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


batch = int(sys.argv[1]) if len(sys.argv) > 1 else 128
torch.manual_seed(3)
base = models.ResNet18().cuda()
x = torch.randn(batch, 3, 32, 32, device="cuda")
y = torch.randint(0, 10, (batch,), device="cuda")
grads = []
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1
for fuse in (False, True, False):
    PF.set_dual_bn_fuse(fuse)
    m = copy.deepcopy(base)
    for _ in range(iters):
        for p in m.parameters():
            p.grad = None
        PF.cross_entropy(m(x), y).backward()
    torch.cuda.synchronize()
    grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
for n, g0 in grads[0].items():
    print(f"{n:40s} fused {rel(grads[1][n], g0):.4f}  rerun {rel(grads[2][n], g0):.4f}")
