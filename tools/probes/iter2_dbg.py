"""Is a second forward/backward of the same model (no optimizer step) reproducible? Compares two
fresh copies run identically, under different gradient-reset styles."""
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


def run(style, iters=2):
    m = copy.deepcopy(base)
    losses = []
    for i in range(iters):
        if style == "none":
            for p in m.parameters():
                p.grad = None
        elif style == "zero" and i > 0:
            for p in m.parameters():
                p.grad.zero_()
        out = m(x)
        loss = PF.cross_entropy(out, y)
        loss.backward()
        torch.cuda.synchronize()
        losses.append(loss.item())
    return losses, {n: p.grad.detach().clone() for n, p in m.named_parameters()}, out.detach().float()


run("none", 1)   # autotune / warm-up
for style in ("none", "zero"):
    la, ga, oa = run(style)
    lb, gb, ob = run(style)
    worst = max(((rel(gb[n], g0), n) for n, g0 in ga.items()))
    print(style, "losses", la, lb, "logits rel", rel(ob, oa), "worst grad", worst)
l1, g1, o1 = run("none", 1)
l2, g2, o2 = run("none", 2)
print("iter1 vs iter2 logits rel", rel(o2, o1), "losses", l1, l2)
