#!/usr/bin/env python3
"""Squeeze-excite kernels at a model's own SE shapes: per-call forward / backward time of the
split path (pool, row-dot, col-dot, scale | ds, row-dot, col-dot, param, dx) against the fused
path (pool+MLP, scale | ds+MLP data, param, dx), plus their max differences.

  python tools/se_bench.py [--model EfficientNetB0] [--batch 128] [--reps 50]  (GPU)
Prints one JSON line per shape and a total line."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def shapes(model_name, batch):
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.nn import functional as NF
    from pytorch_cifar_amd.ops.functional import ACT

    seen = []
    orig = NF.squeeze_excite

    def rec(x, w1, b1, w2, b2, act):
        seen.append((tuple(x.shape), w1.shape[0], ACT[act]))
        return orig(x, w1, b1, w2, b2, act)

    NF.squeeze_excite = rec
    try:
        net = models.MODEL_REGISTRY[model_name]().cuda().train()
        with torch.no_grad():
            net(torch.randn(batch, 3, 32, 32, device="cuda"))
    finally:
        NF.squeeze_excite = orig
    return seen


def time_it(fn, reps):
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
    ap.add_argument("--model", default="EfficientNetB0")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    from pytorch_cifar_amd import _native

    C_ = _native.lib()
    tot = {0: [0.0, 0.0], 1: [0.0, 0.0]}
    for (N, C, H, W), R, act in shapes(args.model, args.batch):
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(N, H, W, C, device="cuda", generator=g).to(torch.bfloat16)
        dout = torch.randn(N, H, W, C, device="cuda", generator=g).to(torch.bfloat16)
        w1 = torch.randn(R, C, device="cuda", generator=g) * 0.1
        w2 = torch.randn(C, R, device="cuda", generator=g) * 0.1
        b1 = torch.randn(R, device="cuda", generator=g) * 0.1
        b2 = torch.randn(C, device="cuda", generator=g) * 0.1
        w2t = w2.t().contiguous()
        row = {"N": N, "HW": H * W, "C": C, "R": R}
        res = {}
        for mode in (0, 1):
            C_.se_fused_mode(mode)
            fwd = C_.se_forward(x, w1, b1, w2, b2, act, w2t)
            bufs = [torch.zeros(R * C, device="cuda"), torch.zeros(R, device="cuda"),
                    torch.zeros(R * C, device="cuda"), torch.zeros(C, device="cuda")]
            bwd = C_.se_backward(dout, x, fwd[1], fwd[2], fwd[3], w1, w2, act, *bufs, True, True, w2t)
            res[mode] = (fwd, bwd)
            tf = time_it(lambda: C_.se_forward(x, w1, b1, w2, b2, act, w2t), args.reps)
            tb = time_it(lambda: C_.se_backward(dout, x, fwd[1], fwd[2], fwd[3], w1, w2, act,
                                                *bufs, True, True, w2t), args.reps)
            row[f"fwd{mode}_us"], row[f"bwd{mode}_us"] = round(tf, 1), round(tb, 1)
            tot[mode][0] += tf
            tot[mode][1] += tb
        (f0, b0), (f1, b1_) = res[0], res[1]
        row["max_out_diff"] = float((f0[0].float() - f1[0].float()).abs().max())
        row["max_dx_diff"] = float((b0[0].float() - b1_[0].float()).abs().max())
        print(json.dumps(row), flush=True)
    C_.se_fused_mode(-1)
    print(json.dumps({"total_fwd_split_us": round(tot[0][0], 1), "total_bwd_split_us": round(tot[0][1], 1),
                      "total_fwd_fused_us": round(tot[1][0], 1), "total_bwd_fused_us": round(tot[1][1], 1)}))


if __name__ == "__main__":
    main()
