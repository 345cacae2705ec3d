"""BatchNorm statistics with a large per-channel mean against a small spread (the E[x^2] - E[x]^2
cancellation case) through the production producer -> consumer chain: the conv epilogue adds the
per-channel partial sums (slab rows on the first call, the sharded accumulator once the BN has
linked to its conv; ordered slab + finalize in deterministic mode) and the BN folds them.

The conv is an identity (1x1, or a 3x3 with only the centre tap), so its bf16 output equals the
bf16 input exactly and the oracle is fp64 BatchNorm of that very tensor (reference
models/resnet.py:25, ``nn.BatchNorm2d`` train semantics: biased batch variance for the output,
unbiased for ``running_var``, momentum 0.1).

Activations are stored in bf16 (8 significant bits): at a mean of 100 the representable spacing is
0.5, so a spread below ~0.5 (the round-3 review's std 0.05) is quantised away before any
statistic is taken. The test therefore uses mean/std ratios of 50-200 with std >= 0.5, where the
data survives bf16 and the naive fp32 E[x^2] - E[x]^2 loses 1e-3 to 1e-1 of the variance.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _identity_conv(C, k):
    from pytorch_cifar_amd import nn as pnn

    conv = pnn.Conv2d(C, C, kernel_size=k, padding=k // 2, bias=False)
    with torch.no_grad():
        w = torch.zeros(C, C, k, k)
        w[torch.arange(C), torch.arange(C), k // 2, k // 2] = 1.0
        conv.weight.copy_(w)
    return conv


def _ref_bn(x64, rm, rv, steps, momentum=0.1, eps=1e-5):
    mean = x64.mean((0, 2, 3))
    var = x64.var((0, 2, 3), unbiased=False)
    n = x64.numel() / x64.shape[1]
    for _ in range(steps):
        rm = (1 - momentum) * rm + momentum * mean
        rv = (1 - momentum) * rv + momentum * var * n / (n - 1)
    out = (x64 - mean[None, :, None, None]) / torch.sqrt(var + eps)[None, :, None, None]
    return out, rm, rv


@pytest.mark.parametrize("deterministic", [False, True])
@pytest.mark.parametrize("N,C,H,k,mean,std", [
    (256, 128, 16, 1, 100.0, 2.0),     # 1x1: generic implicit GEMM
    (256, 128, 16, 3, 100.0, 1.0),     # 3x3 layer-2 shape: halo kernel / igemm
    (128, 64, 32, 3, 100.0, 2.0),      # 3x3 64-channel layer-1 kernel
    (256, 256, 8, 3, 400.0, 4.0),      # 3x3 layer-3 shape
])
def test_bn_large_mean_small_spread(N, C, H, k, mean, std, deterministic):
    import pytorch_cifar_amd
    from pytorch_cifar_amd import nn as pnn

    torch.manual_seed(3)
    dev = "cuda"
    conv = _identity_conv(C, k).to(dev)
    bn = pnn.BatchNorm2d(C).to(dev)
    conv.train()
    bn.train()
    offs = mean + torch.linspace(-0.1, 0.1, C) * mean
    x = (offs[None, :, None, None] + std * torch.randn(N, C, H, H)).to(dev)
    x = x.bfloat16().float().contiguous(memory_format=torch.channels_last)
    pytorch_cifar_amd.set_deterministic(deterministic)
    try:
        steps = 3          # first call: slab + finalize; later calls: the linked accumulator
        with torch.no_grad():
            for _ in range(steps):
                out = bn(conv(x), act=None)
        torch.cuda.synchronize()
    finally:
        pytorch_cifar_amd.set_deterministic(False)
    x64 = x.double()
    ref, rm, rv = _ref_bn(x64, torch.zeros(C, dtype=torch.float64, device=dev),
                          torch.ones(C, dtype=torch.float64, device=dev), steps)
    err = ((out.double() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, f"normalised output rel err {err:.3e}"
    e_rv = ((bn.running_var.double() - rv).abs() / rv).max().item()
    e_rm = ((bn.running_mean.double() - rm).abs() / rm.abs()).max().item()
    assert e_rv < 1e-2, f"running_var max rel err {e_rv:.3e}"
    assert e_rm < 1e-3, f"running_mean max rel err {e_rm:.3e}"
