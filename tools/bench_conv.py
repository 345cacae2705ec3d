#!/usr/bin/env python3
"""Per-shape conv kernel benchmark: native MFMA fwd/dgrad/wgrad vs stock MIOpen (bf16 NHWC).

Sweeps the tile configurations compiled into conv_mfma.hip (``_C.set_conv_tile``) on the
ResNet-18 conv census and prints TFLOP/s per (shape, pass, config) plus the
MIOpen reference, as JSON lines (one per measurement) and a summary table.

  python tools/bench_conv.py [--batch 1024] [--cfgs -1,0,1,3] [--wcfgs -1,0,3] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (Cin, Cout, H, k, s, p)
RESNET18 = [
    (64, 64, 32, 3, 1, 1),
    (64, 128, 32, 3, 2, 1),
    (128, 128, 16, 3, 1, 1),
    (128, 256, 16, 3, 2, 1),
    (256, 256, 8, 3, 1, 1),
    (256, 512, 8, 3, 2, 1),
    (512, 512, 4, 3, 1, 1),
    (64, 128, 32, 1, 2, 0),
    (8, 64, 32, 3, 1, 1),
]


def timeit(fn, iters):
    for _ in range(3):
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
    ap.add_argument("--cfgs", default="-1,0,1,3,4,5,6,7")
    ap.add_argument("--wcfgs", default="-1,0,3,4,5")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default="")
    ap.add_argument("--splits", default="-1", help="split-K overrides for fwd/dgrad (-1 heuristic, 0 off)")
    a = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    N = a.batch
    rows = []
    torch.manual_seed(0)
    for (Cin, Cout, H, k, s, p) in RESNET18:
        Ho = (H + 2 * p - k) // s + 1
        flops = 2.0 * N * Ho * Ho * Cout * Cin * k * k
        x = torch.randn(N, H, H, Cin, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(Cout, k, k, Cin, device="cuda") * 0.05
        dy = torch.randn(N, Ho, Ho, Cout, device="cuda", dtype=torch.bfloat16)
        wb, wt = C.weight_prep(w, 1, True)
        # reference check of the heuristic config
        C.set_conv_tile(0, -1)
        C.set_conv_tile(1, -1)
        y, _ = C.conv_fwd(x, wb, None, s, p, 1, True)
        xr = x.permute(0, 3, 1, 2).float()
        wr = w.permute(0, 3, 1, 2).bfloat16().float()
        yr = F.conv2d(xr, wr, stride=s, padding=p)
        err = ((y.permute(0, 3, 1, 2).float() - yr).abs().max() / yr.abs().max()).item()
        shape = f"{Cin}->{Cout} k{k}s{s} @{H}"
        n_ig = 0
        for sp in [int(v) for v in a.splits.split(",")]:
            C.set_conv_tile(2, sp)
            for cfg in [int(c) for c in a.cfgs.split(",")]:
                C.set_conv_tile(0, cfg)
                tf = timeit(lambda: C.conv_fwd(x, wb, None, s, p, 1, True), a.iters)
                td = timeit(lambda: C.conv_dgrad(dy, wt, H, H, s, p, 1), a.iters) if Cin % 8 == 0 and Cin >= 16 else float("nan")
                rows.append(dict(shape=shape, pass_="fwd", cfg=cfg, split=sp, us=tf * 1e6, tflops=flops / tf / 1e12, err=err))
                rows.append(dict(shape=shape, pass_="dgrad", cfg=cfg, split=sp, us=td * 1e6, tflops=flops / td / 1e12))
                n_ig += 2
        C.set_conv_tile(0, -1)
        C.set_conv_tile(2, -1)
        for cfg in [int(c) for c in a.wcfgs.split(",")]:
            C.set_conv_tile(1, cfg)
            tw = timeit(lambda: C.conv_wgrad(x, dy, k, k, s, p, 1, None), a.iters)
            rows.append(dict(shape=shape, pass_="wgrad", cfg=cfg, us=tw * 1e6, tflops=flops / tw / 1e12))
        C.set_conv_tile(1, -1)
        # stock MIOpen bf16 channels_last
        xm = x.permute(0, 3, 1, 2).requires_grad_(True)
        wm = w.permute(0, 3, 1, 2).bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
        dym = dy.permute(0, 3, 1, 2)
        tmf = timeit(lambda: F.conv2d(xm, wm, stride=s, padding=p), a.iters)
        out = F.conv2d(xm, wm, stride=s, padding=p)
        tmb = timeit(lambda: torch.autograd.grad(out, (xm, wm), dym, retain_graph=True), a.iters)
        rows.append(dict(shape=shape, pass_="miopen_fwd", cfg=None, us=tmf * 1e6, tflops=flops / tmf / 1e12))
        rows.append(dict(shape=shape, pass_="miopen_bwd(d+w)", cfg=None, us=tmb * 1e6, tflops=2 * flops / tmb / 1e12))
        for r in rows[-(n_ig + len(a.wcfgs.split(",")) + 2):]:
            print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
