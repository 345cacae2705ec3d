#!/usr/bin/env python3
"""Time the native BatchNorm backward (reduce + finalize + apply) and statistics kernels on the
EfficientNet-B0 / ResNet-18 activation shapes, one shape at a time, as hipGraph replays (device
time per call; run under ``rocprofv3 --kernel-trace --stats`` for the per-kernel split).

  python tools/probes/bn_shapes.py [--iters 50]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

SHAPES = [  # N, H, C, act (2 = swish, 1 = relu)
    (128, 32, 96, 2), (128, 16, 144, 2), (128, 8, 240, 2), (128, 4, 480, 2), (128, 4, 672, 2),
    (128, 2, 1152, 2), (128, 32, 64, 1), (1024, 4, 512, 1), (1024, 32, 64, 1),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from pytorch_cifar_amd import _native

    C_ = _native.lib()
    print("| N x H x H x C | act | bwd us | stats us |\n|---|---:|---:|---:|")
    for N, H, C, act in SHAPES:
        y = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
        dout = torch.randn_like(y)
        g, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        aux = C_.bn_finalize(C_.bn_stats(y), float(N * H * H), g, b, rm, rv, None, 0.1, 1e-5, True,
                             False)
        out, mask = C_.bn_apply(y, aux, None, None, None, act, act == 1)
        m = mask if (mask is not None and mask.numel()) else None

        def bwd():
            C_.bn_backward(dout, None if m is not None else out, m, y, aux, g, None, None, None, act,
                           True, False, None, None, None, None)

        def stats():
            C_.bn_stats(y)

        res = []
        for fn in (bwd, stats):
            # captured in a hipGraph of `iters` calls: device time per call, no host overhead
            fn()
            torch.cuda.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(a.iters):
                    fn()
            graph.replay()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            graph.replay()
            e.record()
            torch.cuda.synchronize()
            res.append(s.elapsed_time(e) / a.iters * 1e3)
        print(f"| {N}x{H}x{H}x{C} | {act} | {res[0]:.1f} | {res[1]:.1f} |", flush=True)


if __name__ == "__main__":
    main()
