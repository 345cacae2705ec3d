#!/usr/bin/env python3
"""Where a c64 tile's cycles go: per-wave shader-clock stamps (tile start after the barrier,
K-loop end, epilogue end) from the PROF instantiation of conv3x3_c64_kernel; prints medians.

  python tools/c64_stamps.py [--batch 1024] [--pass fwd|dgrad]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--pass", dest="pass_", default="fwd")
    a = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    N, H = a.batch, 32
    x = torch.randn(N, H, H, 64, device="cuda").to(torch.bfloat16)
    w = torch.randn(64, 3, 3, 64, device="cuda") * 0.05
    wb, wt = C.weight_prep(w, 1, True)
    grid = C.c64_grid_size(N, H)
    prof = torch.zeros(grid * 4 * 16 * 4, dtype=torch.int64, device="cuda")
    run = (lambda: C.conv_fwd(x, wb, None, 1, 1, 1, True)) if a.pass_ == "fwd" else \
        (lambda: C.conv_dgrad(x, wt, H, H, 1, 1, 1))
    run()
    torch.cuda.synchronize()
    C.c64_set_prof(prof)
    run()
    torch.cuda.synchronize()
    C.c64_set_prof(None)
    st = prof.view(grid, 4, 16, 4).cpu()
    tiles = (N * H // 8 + grid - 1) // grid
    nt = min(tiles, 16)
    k = (st[:, :, :nt, 1] - st[:, :, :nt, 0]).flatten().float()
    e = (st[:, :, :nt, 2] - st[:, :, :nt, 1]).flatten().float()
    gap = (st[:, :, 1:nt, 0] - st[:, :, :nt - 1, 2]).flatten().float()
    tot = (st[:, :, nt - 1, 2] - st[:, :, 0, 0]).flatten().float() / max(1, nt - 1)
    print(f"grid {grid}, tiles/block {tiles}; cycles per tile (median over waves x tiles):")
    print(f"  K loop (288 MFMA = 4608 cyc at 16/MFMA): {k.median():8.0f}  (p10 {k.quantile(.1):.0f}, p90 {k.quantile(.9):.0f})")
    print(f"  epilogue:                                {e.median():8.0f}")
    print(f"  barrier + halo wait (to next tile):      {gap.median():8.0f}  (p90 {gap.quantile(.9):.0f})")
    print(f"  total per tile:                          {tot.median():8.0f}")


if __name__ == "__main__":
    main()
