#!/usr/bin/env python3
"""1x1-conv GEMMs of ResNet-50/101/152 at a batch: the native implicit-GEMM forward (with its
BN-statistics epilogue) and dgrad (plain) against torch.mm (hipBLASLt) on the same operands.
  python tools/gemm1x1_probe.py [--batch 1024]   (GPU)"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def t(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    B = args.batch
    for hw, cin, cout in [(32, 256, 64), (32, 64, 256), (16, 512, 128), (16, 128, 512),
                          (8, 1024, 256), (8, 256, 1024), (4, 2048, 512), (4, 512, 2048)]:
        M = B * hw * hw
        x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
        dy = torch.randn(B, hw, hw, cout, device="cuda").to(torch.bfloat16)
        w = (torch.randn(cout, 1, 1, cin, device="cuda") * 0.05)
        wb, wt = C.weight_prep(w, 1, True)
        f_nat = t(lambda: C.conv_fwd(x, wb, None, 1, 0, 1, True))
        d_nat = t(lambda: C.conv_dgrad(dy, wt, hw, hw, 1, 0, 1))
        x2, w2 = x.view(M, cin), wb.view(cout, cin)
        f_mm = t(lambda: torch.mm(x2, w2.t()))
        d_mm = t(lambda: torch.mm(dy.view(M, cout), w2))
        gf = 2.0 * M * cin * cout / 1e9
        print(json.dumps({"hw": hw, "cin": cin, "cout": cout, "M": M, "gflop": round(gf, 1),
                          "fwd_native_us": round(f_nat, 1), "fwd_mm_us": round(f_mm, 1),
                          "dgrad_native_us": round(d_nat, 1), "dgrad_mm_us": round(d_mm, 1)}), flush=True)


if __name__ == "__main__":
    main()
