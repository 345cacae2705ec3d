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
