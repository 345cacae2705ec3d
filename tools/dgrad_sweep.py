#!/usr/bin/env python3
"""Per-variant timing of the stride-1 3x3 dgrad vs the forward on the ResNet-18 layer shapes:
plain / + fused BN reduce / + BN + addend, for a list of tile configs (one process).

  python tools/dgrad_sweep.py [--batch 1024] [--cfgs 3,12,20,21,30]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--cfgs", default="3,12,20,21,30")
    ap.add_argument("--shapes", default="64x32,128x16,256x8,512x4")
    ap.add_argument("--relu", default="", help="x / dy / xdy: zero the negative half (ReLU-like)")
    a = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    cfgs = [int(c) for c in a.cfgs.split(",")]
    for shp in a.shapes.split(","):
        ch, h = map(int, shp.split("x"))
        N = a.batch
        x = torch.randn(N, h, h, ch, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(ch, 3, 3, ch, device="cuda") * 0.05
        dy = torch.randn(N, h, h, ch, device="cuda", dtype=torch.bfloat16)
        add = torch.randn_like(x)
        y = torch.randn_like(x)
        mask = torch.randint(0, 256, (x.numel() // 8,), device="cuda", dtype=torch.uint8)
        aux = torch.cat([torch.zeros(ch, device="cuda"), torch.ones(ch, device="cuda")])
        R = 16
        acc = torch.zeros(R * 2 * ch, device="cuda")
        if "x" in a.relu:
            x = torch.relu(x)
        if "dy" in a.relu:
            dy = torch.relu(dy)
        wb, wt = C.weight_prep(w, 1, True)
        fl = 2.0 * N * h * h * ch * ch * 9
        for cfg in cfgs:
            C.set_conv_tile(0, cfg)
            row = []
            try:
                row.append(("fwd", timeit(lambda: C.conv_fwd(x, wb, None, 1, 1, 1, True))))
                row.append(("dg", timeit(lambda: C.conv_dgrad(dy, wt, h, h, 1, 1, 1, None))))
                row.append(("dg+add", timeit(lambda: C.conv_dgrad(dy, wt, h, h, 1, 1, 1, add))))
                row.append(("dg+bn", timeit(lambda: C.conv_dgrad_bn(dy, wt, h, h, 1, 1, 1, None, y, mask, aux, acc, R))))
                row.append(("dg+bn+add", timeit(lambda: C.conv_dgrad_bn(dy, wt, h, h, 1, 1, 1, add, y, mask, aux, acc, R))))
            except RuntimeError as ex:
                row.append(("err", str(ex)[:60]))
            txt = "  ".join(f"{k} {v:7.1f}us ({fl / v / 1e6:4.0f}TF)" if isinstance(v, float) else f"{k} {v}"
                            for k, v in row)
            print(f"{ch}x{h} cfg {cfg:2d}: {txt}", flush=True)
        C.set_conv_tile(0, -1)


if __name__ == "__main__":
    main()
