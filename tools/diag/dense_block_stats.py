"""One DenseNet block, slab with / without the statistics cache: per-BN running-stat and
gradient differences (diagnostic for the cache wiring)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from pytorch_cifar_amd.models.densenet import Bottleneck, Transition, dense_block  # noqa: E402
from pytorch_cifar_amd.nn import Sequential  # noqa: E402
from pytorch_cifar_amd.ops import functional as OF  # noqa: E402

torch.manual_seed(0)
c0, g, L = 64, 32, int(sys.argv[1]) if len(sys.argv) > 1 else 3


class Block(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.dense = Sequential(*[Bottleneck(c0 + i * g, g) for i in range(L)])
        self.trans = Transition(c0 + L * g, 64)

    def forward(self, x):
        return self.trans(dense_block(self.dense, x))


m0 = Block().cuda().to(memory_format=torch.channels_last)
x = torch.randn(8, c0, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
gy = torch.randn(8, 64, 8, 8, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
res = {}
for st in (False, True):
    OF._SLAB_STATS = st
    m = copy.deepcopy(m0)
    xi = x.clone().requires_grad_(True)
    y = m(xi)
    y.backward(gy)
    torch.cuda.synchronize()
    res[st] = (y.float(), xi.grad.float(), {n: b.clone() for n, b in m.named_buffers()},
               {n: p.grad.float().clone() for n, p in m.named_parameters()})


def r(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-9)).item()


print("out", r(res[True][0], res[False][0]), "dx", r(res[True][1], res[False][1]))
for n in res[False][2]:
    if "running" in n:
        print("buf %-28s %.3e" % (n, r(res[True][2][n], res[False][2][n])))
for n in res[False][3]:
    print("grad %-28s %.3e" % (n, r(res[True][3][n], res[False][3][n])))
