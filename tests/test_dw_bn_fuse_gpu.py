"""BN(+ReLU/swish) applied inside the depthwise consumer (ops.functional.bn_act_dwconv,
csrc/dwconv.hip input transform): forward output, BN running statistics and every gradient
(input, BN gamma/beta, depthwise weight) against the unfused native path (BN apply pass, plain
depthwise) and against fp32 torch, training mode, two steps (slab statistics, then the producer's
sharded accumulator). Shapes: MobileNetV2 / EfficientNet-B0 / ShuffleNetV2 depthwise layers."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _block(Cin, C, k, s):
    from pytorch_cifar_amd import nn as pnn

    torch.manual_seed(0)
    conv1 = pnn.Conv2d(Cin, C, kernel_size=1, bias=False)
    bn1 = pnn.BatchNorm2d(C)
    conv2 = pnn.Conv2d(C, C, kernel_size=k, stride=s, padding=k // 2, groups=C, bias=False)
    with torch.no_grad():
        bn1.weight.uniform_(0.5, 1.5)
        bn1.bias.uniform_(-0.2, 0.2)
    return torch.nn.ModuleList([conv1, bn1, conv2]).cuda()


def _run(m, x, act, fused):
    from pytorch_cifar_amd.ops import functional as OF

    conv1, bn1, conv2 = m
    prev = OF._DW_IN_FUSE
    OF._DW_IN_FUSE = fused
    try:
        outs = []
        for it in range(2):
            for p in m.parameters():
                p.grad = None
            xi = x[it].clone().requires_grad_(True)
            y = OF.bn_act_dwconv(bn1, conv1(xi), act, conv2)
            g = torch.randn(y.shape, generator=torch.Generator(device="cuda").manual_seed(it), device="cuda")
            y.float().backward(g)
            torch.cuda.synchronize()
            outs.append((y.float(), xi.grad.float(), {n: p.grad.float().clone() for n, p in m.named_parameters()}))
        return outs, (bn1.running_mean.clone(), bn1.running_var.clone())
    finally:
        OF._DW_IN_FUSE = prev


def _ref(m, x, act):
    conv1, bn1, conv2 = [copy.deepcopy(t).float() for t in m]
    outs = []
    for it in range(2):
        xi = x[it].clone().float().requires_grad_(True)
        z = F.batch_norm(F.conv2d(xi, conv1.weight), bn1.running_mean, bn1.running_var, bn1.weight,
                         bn1.bias, True, 0.1, bn1.eps)
        z = F.relu(z) if act == "relu" else z * torch.sigmoid(z)
        y = F.conv2d(z, conv2.weight, stride=conv2.stride, padding=conv2.padding, groups=conv2.groups)
        g = torch.randn(y.shape, generator=torch.Generator(device="cuda").manual_seed(it), device="cuda")
        params = [conv1.weight, bn1.weight, bn1.bias, conv2.weight]
        grads = torch.autograd.grad(y, [xi] + params, g)
        outs.append((y, grads[0], dict(zip(["0.weight", "1.weight", "1.bias", "2.weight"], grads[1:]))))
    return outs, (bn1.running_mean, bn1.running_var)


@pytest.mark.parametrize("Cin,C,H,k,s,act", [
    (24, 144, 32, 3, 1, "relu"),     # MobileNetV2 stage 2
    (32, 192, 16, 3, 2, "relu"),     # MobileNetV2 downsample
    (40, 240, 8, 5, 1, "swish"),     # EfficientNet-B0 k5
    (112, 672, 4, 5, 2, "swish"),    # EfficientNet-B0 k5 s2
])
def test_bn_act_dwconv_matches_unfused_and_fp32(Cin, C, H, k, s, act):
    torch.manual_seed(1)
    x = [torch.randn(16, Cin, H, H, device="cuda").contiguous(memory_format=torch.channels_last)
         for _ in range(2)]
    m_f = _block(Cin, C, k, s)
    m_u = copy.deepcopy(m_f)
    m_r = copy.deepcopy(m_f)
    fused, rs_f = _run(m_f, x, act, True)
    unfused, rs_u = _run(m_u, x, act, False)
    ref, rs_r = _ref(m_r, x, act)
    for it in range(2):
        (yf, gxf, gpf), (yu, gxu, gpu_), (yr, gxr, gpr) = fused[it], unfused[it], ref[it]
        # the fused transform rounds act(BN(y)) to bf16 exactly as the apply pass stores it
        assert rel(yf, yu) < 2e-3, (it, rel(yf, yu))
        assert rel(yf, yr) < 2e-2, (it, rel(yf, yr))
        assert rel(gxf, gxr) <= 1.5 * rel(gxu, gxr) + 5e-3, (it, rel(gxf, gxr), rel(gxu, gxr))
        for n in gpr:
            assert rel(gpf[n], gpr[n]) <= 1.5 * rel(gpu_[n], gpr[n]) + 5e-3, \
                (it, n, rel(gpf[n], gpr[n]), rel(gpu_[n], gpr[n]))
    for a, b in zip(rs_f, rs_r):
        assert rel(a, b) < 1e-2
    for a, b in zip(rs_f, rs_u):
        assert rel(a, b) < 1e-3
