#!/usr/bin/env python3
"""Microbenchmark of the narrow-K 1x1 forward shapes (MobileNetV2 / EfficientNet-B0 expand convs):
us per call of C.conv_fwd with slab statistics, and the bytes floor at 6 TB/s. Run once per
kernel variant (PCA_CONV_NK=0: generic igemm; PCA_NK_STG=0/1: direct / LDS-staged stores)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from pytorch_cifar_amd import _native

    C = _native.lib()
    tag = sys.argv[1] if len(sys.argv) > 1 else ""
    for N, H, Cin, Cout in [(1024, 32, 16, 96), (1024, 32, 24, 144), (1024, 16, 32, 192),
                            (1024, 16, 40, 240), (128, 32, 16, 96), (128, 16, 24, 144),
                            (128, 16, 40, 240)]:
        x = torch.randn(N, H, H, Cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(Cout, 1, 1, Cin, device="cuda") * 0.1
        wb, _ = C.weight_prep(w, 1, False)
        for _ in range(3):
            C.conv_fwd(x, wb, None, 1, 0, 1, True)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        a.record()
        for _ in range(it):
            C.conv_fwd(x, wb, None, 1, 0, 1, True)
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / it
        mb = N * H * H * (Cin + Cout) * 2 / 1e6
        print(json.dumps({"tag": tag, "shape": [N, H, Cin, Cout], "us": round(us, 1),
                          "floor_us": round(mb / 6e6 * 1e6 / 1e0 / 1e0, 1), "MB": round(mb, 1)}))


if __name__ == "__main__":
    main()
