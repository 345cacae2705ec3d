#!/usr/bin/env python3
"""Time every weight-gradient autotune candidate (config, split) on the ResNet-18 conv census.

For each shape prints the candidates sorted by time (TFLOP/s), the untuned heuristic and what
the autotuner would record, as JSON lines. Split encoding (conv_mfma.hip wgrad_tune_candidates):
-1 occupancy-derived plan, >= 1 forced split count with fp32 atomics, <= -2 fixed slab count.

  python tools/wgrad_sweep.py [--batch 128] [--iters 20] [--top 6]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench_conv import RESNET18, timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--top", type=int, default=6)
    args = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    N = args.batch
    for Cin, Cout, H, k, s, p in RESNET18:
        if Cin < 64:
            continue
        Ho = (H + 2 * p - k) // s + 1
        x = torch.randn(N, H, H, Cin, device="cuda").to(torch.bfloat16)
        dy = torch.randn(N, Ho, Ho, Cout, device="cuda").to(torch.bfloat16)
        flop = 2.0 * N * Ho * Ho * Cout * Cin * k * k
        res = []
        cands = C.wgrad_candidates(N, H, H, Cin, Cout, k, k, s, p, 1)
        try:
            for cfg, split in [(-1, -1)] + list(cands):
                C.conv_trial(1, cfg, split)
                t = timeit(lambda: C.conv_wgrad(x, dy, k, k, s, p, 1, None), args.iters)
                res.append((t, cfg, split))
        finally:
            C.conv_trial(1, -1, -1)
        heur = res[0]
        res = sorted(res[1:])
        for t, cfg, split in [heur] + res[: args.top]:
            print(json.dumps({"shape": f"{Cin}->{Cout} k{k}s{s} @{H}", "batch": N, "cfg": cfg,
                              "split": split, "us": round(t * 1e6, 2),
                              "tflops": round(flop / t / 1e12, 1),
                              "heuristic": (cfg, split) == (-1, -1)}), flush=True)


if __name__ == "__main__":
    main()
