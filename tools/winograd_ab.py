#!/usr/bin/env python3
"""Winograd F(2x2,3x3) candidate vs the native implicit-GEMM 3x3 kernels, ResNet-18 3x3/s1 shapes:
per-stage time of the unfused Winograd (input transform, filter transform, 16 batched GEMMs on
hipBLASLt, output transform) against the autotuned native forward, plus relative error vs fp32.
One JSON line per shape (README "Winograd: measured and rejected").

  python tools/winograd_ab.py [--batch 1024]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    a = ap.parse_args()
    from pytorch_cifar_amd import _native
    from pytorch_cifar_amd.ops import winograd as wg

    C = _native.lib()
    N = a.batch
    for (Cin, Cout, H) in [(64, 64, 32), (128, 128, 16), (256, 256, 8), (512, 512, 4)]:
        torch.manual_seed(0)
        x = torch.randn(N, H, H, Cin, device="cuda").bfloat16()
        w = torch.randn(Cout, Cin, 3, 3, device="cuda") * (2.0 / (Cin * 9)) ** 0.5
        wb, _ = C.weight_prep(w.permute(0, 2, 3, 1).contiguous(), 1, False)
        ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.bfloat16().float(), padding=1).permute(0, 2, 3, 1)
        y_n, _ = C.conv_fwd(x, wb, None, 1, 1, 1, True)
        y_w = wg.conv3x3_winograd(x, w)
        err = lambda y: ((y.float() - ref).norm() / ref.norm()).item()
        V = wg.input_transform(x)
        U = wg.filter_transform(w)
        M = wg.batched_gemm(V, U)
        row = dict(shape=f"{Cin}->{Cout} @{H}", batch=N,
                   native_us=timeit(lambda: C.conv_fwd(x, wb, None, 1, 1, 1, True)),
                   wino_input_us=timeit(lambda: wg.input_transform(x)),
                   wino_filter_us=timeit(lambda: wg.filter_transform(w)),
                   wino_gemm_us=timeit(lambda: wg.batched_gemm(V, U)),
                   wino_output_us=timeit(lambda: wg.output_transform(M, N, H, H)),
                   err_native=err(y_n), err_wino=err(y_w),
                   transformed_bytes=V.numel() * 2 + M.numel() * M.element_size())
        row["wino_total_us"] = row["wino_input_us"] + row["wino_gemm_us"] + row["wino_output_us"]
        if C.winograd_applicable(N, H, H, Cin, Cout):
            # the fused kernel (csrc/winograd.hip), with its BN-statistics epilogue like the
            # native forward it would replace; the filter transform is timed apart (it would run
            # once per step in the fused optimizer launch)
            wp = w.permute(0, 2, 3, 1).contiguous()
            Uf = C.winograd_filter(wp)
            y_f, _ = C.winograd_fwd(x, Uf, True)
            row.update(fused_us=timeit(lambda: C.winograd_fwd(x, Uf, True)),
                       fused_filter_us=timeit(lambda: C.winograd_filter(wp)), err_fused=err(y_f))
            row["fused_vs_native"] = row["fused_us"] / row["native_us"]
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)


if __name__ == "__main__":
    main()
