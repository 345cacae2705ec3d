#!/usr/bin/env python3
"""Time every wgrad autotune candidate (cfg, split) of one conv geometry (HIP events), sorted.

  python tools/wgrad_sweep.py --batch 128 --cin 512 --cout 512 --h 4 [--top 12]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--cin", type=int, default=512)
    ap.add_argument("--cout", type=int, default=512)
    ap.add_argument("--h", type=int, default=4)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--s", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    p = a.k // 2
    Ho = (a.h + 2 * p - a.k) // a.s + 1
    N = a.batch
    x = torch.randn(N, a.h, a.h, a.cin, device="cuda").to(torch.bfloat16)
    dy = torch.randn(N, Ho, Ho, a.cout, device="cuda").to(torch.bfloat16)
    dw = torch.zeros(a.cout, a.k, a.k, a.cin, device="cuda")
    res = []
    for cfg, split in C.wgrad_candidates(N, a.h, a.h, a.cin, a.cout, a.k, a.k, a.s, p, 1):
        C.conv_trial(1, cfg, split)
        for _ in range(3):
            C.conv_wgrad(x, dy, a.k, a.k, a.s, p, 1, dw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            C.conv_wgrad(x, dy, a.k, a.k, a.s, p, 1, dw)
        e1.record()
        torch.cuda.synchronize()
        res.append((e0.elapsed_time(e1) * 1e3 / a.iters, cfg, split))
    C.conv_trial(1, -1, -1)
    res.sort()
    flops = 2 * N * Ho * Ho * a.cout * a.cin * a.k * a.k
    for us, cfg, split in res[:a.top]:
        print(json.dumps({"shape": [N, a.cin, a.cout, a.h, a.k, a.s], "cfg": cfg, "split": split,
                          "us": round(us, 1), "tflops": round(flops / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
