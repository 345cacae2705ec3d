"""Winograd F(2x2, 3x3) for the 3x3 / stride-1 / pad-1 convolutions (BASELINE
north star "implicit-GEMM / Winograd"; reference models/resnet.py:23-27, 98.9 % of ResNet-18's
MACs).

Two forms:

* :func:`conv3x3_winograd_fused` — the fused gfx950 kernel (csrc/winograd.hip): input transform
  in registers per 4x4 patch, the 16 per-point GEMMs on MFMA out of LDS, output transform and the
  BatchNorm-statistics epilogue in registers; the filter transform U = G g G^T is one small native
  launch from the fp32 master. Measured per call against the tuned native direct kernels by
  ``tools/winograd_ab.py`` (README records the decision).
* the unfused stock-op harness below (einsum / bmm on hipBLASLt; also the CPU reference): input
  transform V = B^T d B of every 4x4 input tile (stride 2), filter transform
U = G g G^T, 16 batched GEMMs M = V U over the transform points (bf16 operands, fp32
accumulation), output transform Y = A^T M A. It runs on stock PyTorch ops (einsum / bmm ->
hipBLASLt) so the three stages can be timed separately against the native implicit-GEMM kernels
(tools/winograd_ab.py). The GEMM stage does 16/36 of the direct MACs (2.25x fewer), but unfused
the transformed operands are 4x the activation tensor each way: for ResNet-18 layer 2 at bs1024,
V and M are 268 MB each in bf16 — ~1.1 GB of extra HBM traffic per conv (~200 us at 5.5 TB/s)
against the ~85 us the native halo kernel takes for the whole conv. A fused F(2x2,3x3) kernel
would have to do the transforms in LDS per tile around 16 per-point MFMA GEMMs; the measured
unfused stages bound what such a kernel could save (the GEMM stage alone) and are recorded with
the decision.
"""
from __future__ import annotations

import torch

# F(2x2, 3x3) transform matrices (Lavin & Gray 2016)
_BT = [[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]]
_G = [[1, 0, 0], [0.5, 0.5, 0.5], [0.5, -0.5, 0.5], [0, 0, 1]]
_AT = [[1, 1, 1, 0], [0, 1, -1, -1]]


def _mats(device):
    f = dict(dtype=torch.float32, device=device)
    return torch.tensor(_BT, **f), torch.tensor(_G, **f), torch.tensor(_AT, **f)


def filter_transform(w: torch.Tensor) -> torch.Tensor:
    """w [Cout, Cin, 3, 3] -> U [16, Cin, Cout] (bf16)."""
    _, G, _ = _mats(w.device)
    U = torch.einsum("ik,ockl,jl->ijco", G, w.float(), G)        # [4, 4, Cin, Cout]
    return U.reshape(16, U.shape[2], U.shape[3]).contiguous().to(torch.bfloat16)


def input_transform(x: torch.Tensor) -> torch.Tensor:
    """x NHWC [N, H, W, C] (H, W even) -> V [16, N*(H/2)*(W/2), C] (bf16)."""
    BT, _, _ = _mats(x.device)
    N, H, W, C = x.shape
    xp = torch.nn.functional.pad(x, (0, 0, 1, 1, 1, 1))             # zero pad H and W by 1
    t = xp.unfold(1, 4, 2).unfold(2, 4, 2)                           # [N, H/2, W/2, C, 4, 4]
    V = torch.einsum("ik,nhwckl,jl->ijnhwc", BT, t.float(), BT)      # [4, 4, N, H/2, W/2, C]
    return V.reshape(16, N * (H // 2) * (W // 2), C).to(torch.bfloat16)


def batched_gemm(V: torch.Tensor, U: torch.Tensor) -> torch.Tensor:
    """M [16, P, Cout] = V [16, P, Cin] @ U [16, Cin, Cout] (bf16 in, fp32 accumulate)."""
    return torch.bmm(V, U)


def output_transform(M: torch.Tensor, N: int, H: int, W: int) -> torch.Tensor:
    """M [16, P, Cout] -> y NHWC [N, H, W, Cout] (bf16)."""
    _, _, AT = _mats(M.device)
    Cout = M.shape[-1]
    Mt = M.float().reshape(4, 4, N, H // 2, W // 2, Cout)
    Y = torch.einsum("ik,klnhwc,jl->nhiwjc", AT, Mt, AT)             # [N, H/2, 2, W/2, 2, Cout]
    return Y.reshape(N, H, W, Cout).to(torch.bfloat16)


def conv3x3_winograd(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """3x3 / stride 1 / pad 1 convolution of NHWC ``x`` with ``w`` [Cout, Cin, 3, 3]."""
    N, H, W, _ = x.shape
    assert H % 2 == 0 and W % 2 == 0 and w.shape[2:] == (3, 3)
    return output_transform(batched_gemm(input_transform(x), filter_transform(w)), N, H, W)


def conv3x3_winograd_fused(x: torch.Tensor, w: torch.Tensor, want_stats: bool = False):
    """Fused native Winograd F(2x2,3x3) forward of NHWC bf16 ``x`` with ``w`` [Cout, Cin, 3, 3]
    (any layout; fp32): returns (y NHWC bf16, BN partial sums [rows][2][Cout] or empty)."""
    from .. import _native

    C = _native.lib()
    U = C.winograd_filter(w.float().permute(0, 2, 3, 1).contiguous())
    return C.winograd_fwd(x.contiguous(), U, want_stats)
