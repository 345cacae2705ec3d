#!/usr/bin/env python3
"""Library-GEMM probe: torch.mm (hipBLASLt) bf16 x bf16 -> fp32 at the ResNet-18 weight-gradient
GEMM shapes dW[Cout][9*Cin] = dY^T[Cout][P] x im2col(X)[P][9*Cin], for comparison with the
native implicit-GEMM wgrads (autotune logs)."""
import torch

shapes = [("l4 bs128", 512, 2048, 4608), ("l3 bs128", 256, 8192, 2304), ("l2 bs128", 128, 32768, 1152),
          ("l4 bs1024", 512, 16384, 4608), ("l3 bs1024", 256, 65536, 2304)]
for name, M, K, N in shapes:
    dy = torch.randn(K, M, device="cuda", dtype=torch.bfloat16)
    col = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    f = lambda: torch.mm(dy.t(), col, out_dtype=torch.float32)
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        f()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 50 * 1e3
    print(f"{name:10s} M={M} K={K} N={N}: {us:7.1f} us  {2*M*N*K/us/1e6:7.1f} TFLOP/s  im2col bytes {K*N*2/1e6:.1f} MB", flush=True)
