#!/usr/bin/env python3
"""Depthwise conv kernel bandwidth on the MobileNetV2 / EfficientNet-B0 shapes (forward, dgrad,
wgrad): GB/s of compulsory traffic (x read + y written once).

  python tools/dw_bench.py [--batch 1024]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


SHAPES = [(96, 32, 3, 1), (144, 32, 3, 1), (144, 32, 3, 2), (192, 16, 3, 1), (384, 8, 3, 1),
          (576, 8, 3, 1), (960, 4, 3, 1), (240, 16, 5, 1), (672, 8, 5, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    print("| C x H, k, s | fwd us | GB/s | dgrad us | GB/s | wgrad us |\n|---|---:|---:|---:|---:|---:|")
    for ch, h, k, s in SHAPES:
        p = k // 2
        x = torch.randn(a.batch, h, h, ch, device="cuda", dtype=torch.bfloat16)
        wT = torch.randn(k * k, ch, device="cuda") * 0.1
        y = C.dw_fwd(x, wT, k, k, s, p)
        dy = torch.randn_like(y)
        nb = (x.numel() + y.numel()) * 2
        tf = timeit(lambda: C.dw_fwd(x, wT, k, k, s, p))
        td = timeit(lambda: C.dw_dgrad(dy, wT, h, h, ch, k, k, s, p))
        tw = timeit(lambda: C.dw_wgrad(x, dy, k, k, s, p))
        print(f"| {ch}x{h} k{k} s{s} | {tf * 1e6:.1f} | {nb / tf / 1e9:.0f} | {td * 1e6:.1f} | "
              f"{nb / td / 1e9:.0f} | {tw * 1e6:.1f} |", flush=True)


if __name__ == "__main__":
    main()
