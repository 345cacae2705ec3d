#!/usr/bin/env python3
"""Time the production selection of one conv geometry: forward (+BN stats), dgrad (plain, with
the fused residual addend and BN-backward reduce) and wgrad, with HIP events; prints one JSON line
per pass (us per call, TFLOP/s). Autotuning runs first, as in training.

  python tools/time_conv.py --batch 1024 --cin 64 --cout 64 --h 32 [--passes fwd,dgrad,dgrad_bn,wgrad]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--cin", type=int, default=64)
    ap.add_argument("--cout", type=int, default=64)
    ap.add_argument("--h", type=int, default=32)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--s", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--passes", default="fwd,dgrad,dgrad_bn,wgrad")
    ap.add_argument("--cfg", type=int, default=-1, help="force a fwd/dgrad tile config (-1: autotune)")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    torch.manual_seed(0)
    p = a.k // 2
    Ho = (a.h + 2 * p - a.k) // a.s + 1
    N = a.batch
    x = torch.randn(N, a.h, a.h, a.cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(a.cout, a.k, a.k, a.cin, device="cuda") * 0.05
    dy = torch.randn(N, Ho, Ho, a.cout, device="cuda").to(torch.bfloat16)
    wb, wt = C.weight_prep(w, 1, True)
    C.set_conv_tile(0, a.cfg)
    # BN-backward fusion operands of the layer that produced x (y, 1-bit ReLU mask, mean | istd)
    ybn = torch.randn_like(x)
    mask = torch.randint(0, 256, (x.numel() // 8,), device="cuda", dtype=torch.uint8)
    aux = torch.cat([torch.zeros(a.cin), torch.ones(a.cin)]).cuda()
    add = torch.randn_like(x)
    dw = torch.zeros(a.cout, a.k, a.k, a.cin, device="cuda")
    fns = {
        "fwd": lambda: C.conv_fwd(x, wb, None, a.s, p, 1, True),
        "dgrad": lambda: C.conv_dgrad(dy, wt, a.h, a.h, a.s, p, 1),
        "dgrad_bn": lambda: C.conv_dgrad_bn(dy, wt, a.h, a.h, a.s, p, 1, add, ybn, mask, aux),
        "wgrad": lambda: C.conv_wgrad(x, dy, a.k, a.k, a.s, p, 1, dw),
    }
    macs = N * Ho * Ho * a.cout * a.cin * a.k * a.k
    for name in a.passes.split(","):
        fn = fns[name]
        for _ in range(3):          # autotune + warm-up
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        print(json.dumps({"tag": a.tag, "shape": [N, a.cin, a.cout, a.h, a.k, a.s], "pass": name, "us": round(us, 1),
                          "tflops": round(2 * macs / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
