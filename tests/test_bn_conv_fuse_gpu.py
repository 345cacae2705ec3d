"""BN+ReLU applied inside the consumer 3x3 conv (ops.functional.bn_act_conv: the layer-1 c64
forward transforms its halo in LDS and writes the ReLU mask, the halo weight gradient transforms
its X stages; csrc/conv3x3_c64.hip / conv_halo.hip XF). Training mode, two steps (the producer
conv's slab statistics, then its sharded accumulator: the fused node runs on the second).

Against the unfused native path (BN apply pass + plain c64 conv): the forward output, the BN
running statistics and every gradient to fp32-summation-order tolerance (the statistics are folded
by the finalize kernel instead of the apply kernel's prologue).
Against fp32 torch: the bf16 tolerance of the other zoo tests. Reference: models/resnet.py:47
(conv2(relu(bn1(conv1(x))))) of the reference BasicBlock."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _block():
    from pytorch_cifar_amd import nn as pnn

    torch.manual_seed(0)
    conv1 = pnn.Conv2d(64, 64, kernel_size=3, padding=1, bias=False)
    bn1 = pnn.BatchNorm2d(64)
    conv2 = pnn.Conv2d(64, 64, kernel_size=3, padding=1, bias=False)
    with torch.no_grad():
        bn1.weight.uniform_(0.5, 1.5)
        bn1.bias.uniform_(-0.3, 0.3)
    return torch.nn.ModuleList([conv1, bn1, conv2]).cuda()


def _run(m, xs, fused):
    from pytorch_cifar_amd.nn.modules import _STATS_ATTR
    from pytorch_cifar_amd.ops import functional as OF

    conv1, bn1, conv2 = m
    prev = OF._BN_CONV_FUSE
    OF._BN_CONV_FUSE = fused
    used0 = OF._BN_CONV_USED[0]
    try:
        outs = []
        for it, x in enumerate(xs):
            for p in m.parameters():
                p.grad = None
            xi = x.clone().requires_grad_(True)
            y = OF.bn_act_conv(bn1, conv1(xi), "relu", conv2)
            assert getattr(y, _STATS_ATTR, None) is not None   # conv2's statistics ride along
            g = torch.randn(y.shape, generator=torch.Generator(device="cuda").manual_seed(it),
                            device="cuda")
            y.float().backward(g)
            torch.cuda.synchronize()
            outs.append((y.float(), xi.grad.float(),
                         {n: p.grad.float().clone() for n, p in m.named_parameters()}))
        return outs, (bn1.running_mean.clone(), bn1.running_var.clone()), OF._BN_CONV_USED[0] - used0
    finally:
        OF._BN_CONV_FUSE = prev


def _ref(m, xs):
    conv1, bn1, conv2 = m
    rm, rv = torch.zeros(64, device="cuda"), torch.ones(64, device="cuda")
    outs = []
    for it, x in enumerate(xs):
        w1 = conv1.weight.detach().float().clone().requires_grad_(True)
        w2 = conv2.weight.detach().float().clone().requires_grad_(True)
        ga = bn1.weight.detach().float().clone().requires_grad_(True)
        be = bn1.bias.detach().float().clone().requires_grad_(True)
        xi = x.float().clone().requires_grad_(True)
        z = F.batch_norm(F.conv2d(xi, w1, padding=1), rm, rv, ga, be, True, 0.1, bn1.eps)
        y = F.conv2d(F.relu(z), w2, padding=1)
        g = torch.randn(y.shape, generator=torch.Generator(device="cuda").manual_seed(it),
                        device="cuda")
        y.backward(g)
        outs.append((y, xi.grad, {"0.weight": w1.grad, "1.weight": ga.grad, "1.bias": be.grad,
                                  "2.weight": w2.grad}))
    return outs, (rm, rv)


@pytest.mark.parametrize("N", [16, 128])
def test_bn_act_conv_matches_unfused_and_fp32(N):
    gen = torch.Generator(device="cpu").manual_seed(5)
    xs = [(torch.randn(N, 64, 32, 32, generator=gen) * 1.5 + 0.3).cuda().to(torch.bfloat16)
          .contiguous(memory_format=torch.channels_last) for _ in range(2)]
    mf, mu = _block(), _block()
    of, (rmf, rvf), used = _run(mf, xs, True)
    ou, (rmu, rvu), used_u = _run(mu, xs, False)
    assert used == 1 and used_u == 0, (used, used_u)   # fused on the accumulator step only
    outr, (rmr, rvr) = _ref(_block(), xs)
    for it in range(2):
        (yf, dxf, gf), (yu, dxu, gu), (yr, dxr, gr) = of[it], ou[it], outr[it]
        # (the BN statistics are folded by the finalize kernel instead of the fused apply's
        # prologue: same sums, another fp32 summation order -> last-bit scale / shift changes)
        assert rel(yf, yu) < 1e-3, (it, rel(yf, yu))
        assert rel(dxf, dxu) < 1e-3, (it, rel(dxf, dxu))
        for n in gu:
            assert rel(gf[n], gu[n]) < 1e-3, (it, n, rel(gf[n], gu[n]))
        # vs fp32: as close as the unfused native path (bf16 through two convs + the BN backward)
        assert rel(yf, yr) < 0.02, (it, rel(yf, yr))
        assert rel(dxf, dxr) <= 1.1 * rel(dxu, dxr) + 1e-3 and rel(dxf, dxr) < 0.06, \
            (it, rel(dxf, dxr), rel(dxu, dxr))
        for n in gr:
            ef, eu = rel(gf[n], gr[n]), rel(gu[n], gr[n])
            assert ef <= 1.1 * eu + 1e-3 and ef < 0.06, (it, n, ef, eu)
    assert rel(rmf, rmu) < 1e-5 and rel(rvf, rvu) < 1e-5
    assert rel(rmf, rmr) < 0.01 and rel(rvf, rvr) < 0.01


def test_resnet18_step_uses_bn_conv_fusion():
    """The ResNet-18 layer-1 blocks take the fused node from the second training step on, and the
    step's logits match the unfused path's."""
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.ops import functional as OF
    from pytorch_cifar_amd.ops.functional import cross_entropy

    gen = torch.Generator(device="cpu").manual_seed(2)
    xs = [torch.randn(32, 3, 32, 32, generator=gen).cuda() for _ in range(2)]
    ys = [torch.randint(0, 10, (32,), generator=gen).cuda() for _ in range(2)]
    logits = {}
    for fused in (True, False):
        torch.manual_seed(0)
        net = models.ResNet18().cuda().train()
        prev = OF._BN_CONV_FUSE
        OF._BN_CONV_FUSE = fused
        used0 = OF._BN_CONV_USED[0]
        try:
            for x, y in zip(xs, ys):
                out = net(x)
                cross_entropy(out, y).backward()
            torch.cuda.synchronize()
        finally:
            OF._BN_CONV_FUSE = prev
        logits[fused] = out.float()
        assert OF._BN_CONV_USED[0] - used0 == (2 if fused else 0)
    # (last-bit statistics differences amplified through 18 bf16 layers; a transform bug is O(1))
    assert rel(logits[True], logits[False]) < 0.02, rel(logits[True], logits[False])
