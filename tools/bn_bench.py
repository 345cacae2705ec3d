#!/usr/bin/env python3
"""Bandwidth of the native BatchNorm apply / backward-apply row kernels on ResNet-18 shapes.

Times C.bn_apply (ReLU, +residual, +second BN) and C.bn_backward (masked ReLU, +residual
gradient) on NHWC bf16 activations and reports GB/s of compulsory traffic (every tensor read or
written once, masks at 1 bit per element).

  python tools/bn_bench.py [--batch 1024]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    print("| shape | kernel | us | GB/s |\n|---|---|---:|---:|")
    for ch, hw in ((64, 32), (128, 16), (256, 8), (512, 4)):
        M = a.batch * hw * hw
        T = M * ch * 2
        y = torch.randn(a.batch, hw, hw, ch, device="cuda", dtype=torch.bfloat16)
        r = torch.randn_like(y)
        rm, rv = torch.zeros(ch, device="cuda"), torch.ones(ch, device="cuda")
        g, b = torch.ones(ch, device="cuda"), torch.zeros(ch, device="cuda")
        aux = C.bn_finalize(C.bn_stats(y), float(M), g, b, rm, rv, None, 0.1, 1e-5, True, False)
        out, mask = C.bn_apply(y, aux, None, None, None, 1, True)
        dst = torch.empty_like(y)
        cases = [
            ("copy (stock)", lambda: dst.copy_(y), 2 * T),
            ("copy_rows", lambda: C.copy_rows(y, dst), 2 * T),
            ("apply relu", lambda: C.bn_apply(y, aux, None, None, None, 1, True), 2 * T + T / 16),
            ("apply relu no mask", lambda: C.bn_apply(y, aux, None, None, None, 1, False), 2 * T),
            ("apply none", lambda: C.bn_apply(y, aux, None, None, None, 0, False), 2 * T),
            ("apply +res relu", lambda: C.bn_apply(y, aux, r, None, None, 1, True), 3 * T + T / 16),
            ("apply +bn2 relu", lambda: C.bn_apply(y, aux, None, r, aux, 1, True), 3 * T + T / 16),
            ("bwd relu", lambda: C.bn_backward(r, None, mask, y, aux, g, None, None, None, 1, True,
                                               False, None, None, None, None), 3 * T + T / 16),
            ("bwd relu +dres", lambda: C.bn_backward(r, None, mask, y, aux, g, None, None, None, 1,
                                                     True, True, None, None, None, None),
             4 * T + T / 16),
        ]
        for name, fn, nbytes in cases:
            t = timeit(fn)
            print(f"| {a.batch}x{hw}x{hw}x{ch} | {name} | {t * 1e6:.1f} | {nbytes / t / 1e9:.0f} |")


if __name__ == "__main__":
    main()
