"""Winograd F(2x2,3x3) candidate (ops/winograd.py): numerics against fp32 on the same bf16
operands. CPU at a small shape; GPU at the ResNet-18 census shapes (batch 64).
The measured decision (rejected: unfused transforms cost more HBM traffic than the whole native
conv) is in README; this pins the error bound of the candidate."""
import pytest
import torch
import torch.nn.functional as F


def _case(N, Cin, Cout, H, device):
    from pytorch_cifar_amd.ops.winograd import conv3x3_winograd

    torch.manual_seed(0)
    x = torch.randn(N, H, H, Cin, device=device).bfloat16()
    w = torch.randn(Cout, Cin, 3, 3, device=device) * (2.0 / (Cin * 9)) ** 0.5
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.bfloat16().float(), padding=1).permute(0, 2, 3, 1)
    y = conv3x3_winograd(x, w)
    return ((y.float() - ref).norm() / ref.norm()).item()


def test_winograd_cpu_small():
    # bf16 V / U / M roundings: ~3x the direct bf16 conv's output rounding (1.7e-3)
    assert _case(2, 32, 48, 16, "cpu") < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("Cin,Cout,H", [(64, 64, 32), (128, 128, 16), (256, 256, 8), (512, 512, 4)])
def test_winograd_gpu_census(Cin, Cout, H):
    assert _case(64, Cin, Cout, H, "cuda") < 1.5e-2


@pytest.mark.gpu
@pytest.mark.parametrize("N,Cin,Cout,H", [(64, 64, 64, 32), (64, 128, 128, 16), (64, 256, 256, 8),
                                          (64, 512, 512, 4), (3, 96, 192, 6), (5, 32, 64, 2)])
def test_winograd_fused_kernel(N, Cin, Cout, H):
    """The fused kernel (csrc/winograd.hip) against fp32 F.conv2d on the same bf16 operands, and
    its BN-statistics epilogue against the sums of its own output (partial rows, tail tiles)."""
    from pytorch_cifar_amd.ops.winograd import conv3x3_winograd_fused

    torch.manual_seed(1)
    x = torch.randn(N, H, H, Cin, device="cuda").bfloat16()
    w = torch.randn(Cout, Cin, 3, 3, device="cuda") * (2.0 / (Cin * 9)) ** 0.5
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.bfloat16().float(), padding=1).permute(0, 2, 3, 1)
    y, st = conv3x3_winograd_fused(x, w, want_stats=True)
    torch.cuda.synchronize()
    err = ((y.float() - ref).norm() / ref.norm()).item()
    assert err < 1.2e-2, err
    # the epilogue sums the fp32 outputs, the reference their bf16 roundings: the difference is
    # a random walk of per-element roundings (<= 2^-8 relative each)
    s = st.sum(0)
    yf = y.float().reshape(-1, Cout)
    tol = 4e-3 * yf.abs().sum(0) / (yf.shape[0] ** 0.5) * 4 + 1e-3
    assert ((s[0] - yf.sum(0)).abs() <= tol).all()
    assert ((s[1] - (yf * yf).sum(0)).abs() <= 4e-3 * (yf * yf).sum(0) + 1e-3).all()
