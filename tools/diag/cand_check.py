#!/usr/bin/env python3
"""Numerics of EVERY autotune candidate at production shapes (the autotuner may pick any of them
on a given box): forward (+BN sums), dgrad with the fused residual addend + BN-backward reduce
(slab and sharded-accumulator forms, and the dual-BN third sum), and every wgrad candidate,
against fp32 torch on the same bf16 operands. Prints one line per failing candidate and a
summary; exit status 1 when any candidate is wrong.

  python tools/diag/cand_check.py --batch 1024 [--shapes resnet18]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

# (Cin, Cout, H, k, s, p)
RESNET18 = [
    (64, 64, 32, 3, 1, 1), (64, 128, 32, 3, 2, 1), (128, 128, 16, 3, 1, 1),
    (128, 256, 16, 3, 2, 1), (256, 256, 8, 3, 1, 1), (256, 512, 8, 3, 2, 1),
    (512, 512, 4, 3, 1, 1), (64, 128, 32, 1, 2, 0), (128, 256, 16, 1, 2, 0), (256, 512, 8, 1, 2, 0),
]


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--tol", type=float, default=2e-2)
    ap.add_argument("--skip-wgrad", action="store_true")
    a = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    C.conv_autotune(False)
    N = a.batch
    bad, n_ok = [], 0
    for (Cin, Cout, H, k, s, p) in RESNET18:
        torch.manual_seed(0)
        Ho = (H + 2 * p - k) // s + 1
        x = torch.randn(N, Cin, H, H, device="cuda").bfloat16().float().requires_grad_(True)
        w = (torch.randn(Cout, Cin, k, k, device="cuda") * (2.0 / (Cin * k * k)) ** 0.5).bfloat16().float()
        ref = F.conv2d(x, w, stride=s, padding=p)
        dy = torch.randn_like(ref).bfloat16().float()
        ref.backward(dy)
        x_n = x.detach().permute(0, 2, 3, 1).contiguous().bfloat16()
        dy_n = dy.permute(0, 2, 3, 1).contiguous().bfloat16()
        wb, wt = C.weight_prep(w.permute(0, 2, 3, 1).contiguous(), 1, True)
        ref_y = ref.detach().permute(0, 2, 3, 1)
        ref_dx = x.grad.permute(0, 2, 3, 1)
        # BN(+ReLU) that produced x: y, 1-bit mask, mean | istd; addend
        ybn = torch.randn(N, H, H, Cin, device="cuda").bfloat16()
        ybn2 = torch.randn(N, H, H, Cin, device="cuda").bfloat16()
        m = torch.rand(N, H, H, Cin, device="cuda") > 0.4
        bits = (m.view(-1, 8).to(torch.int32) << torch.arange(8, device="cuda")).sum(1).to(torch.uint8)
        mean, istd = torch.randn(Cin, device="cuda") * 0.1, torch.rand(Cin, device="cuda") + 0.5
        mean2, istd2 = torch.randn(Cin, device="cuda") * 0.1, torch.rand(Cin, device="cuda") + 0.5
        aux = torch.cat([mean, istd]).contiguous()
        aux2 = torch.cat([mean2, istd2]).contiguous()
        add = torch.randn(N, H, H, Cin, device="cuda").bfloat16()
        dxa = (ref_dx + add.float()).bfloat16().float()
        dz = dxa * m
        r_s1 = dz.sum((0, 1, 2))
        r_s2 = (dz * (ybn.float() - mean) * istd).sum((0, 1, 2))
        r_s3 = (dz * (ybn2.float() - mean2) * istd2).sum((0, 1, 2))
        shape = f"{Cin}->{Cout} k{k}s{s} @{H}"
        for kind in (0, 1):
            for cfg, split in C.igemm_candidates(kind, N, H, H, Cin, Cout, k, k, s, p, 1, Ho, Ho):
                C.conv_trial(0, cfg, split)
                try:
                    if kind == 0:
                        y, st = C.conv_fwd(x_n, wb, None, s, p, 1, True)
                        e = [rel(y, ref_y), rel(st[:, 0, :].sum(0), ref_y.sum((0, 1, 2)))]
                        # sharded accumulator form
                        R = 8
                        acc = torch.zeros(R * 2 * Cout, device="cuda")
                        y2, _ = C.conv_fwd(x_n, wb, None, s, p, 1, True, acc, R)
                        e += [rel(y2, ref_y), rel(acc.view(R, 2, Cout)[:, 0].sum(0), ref_y.sum((0, 1, 2))),
                              rel(acc.view(R, 2, Cout)[:, 1].sum(0), (y2.float() ** 2).sum((0, 1, 2)))]
                        tag = "fwd"
                    else:
                        dx = C.conv_dgrad(dy_n, wt, H, H, s, p, 1)
                        e = [rel(dx, ref_dx)]
                        dx2, part = C.conv_dgrad_bn(dy_n, wt, H, H, s, p, 1, add, ybn, bits, aux)
                        e.append(rel(dx2, dxa))
                        if part.numel():
                            e += [rel(part[:, 0].sum(0), r_s1), rel(part[:, 1].sum(0), r_s2)]
                        R = 8
                        acc = torch.zeros(R * 3 * Cin, device="cuda")
                        dx3, part3 = C.conv_dgrad_bn(dy_n, wt, H, H, s, p, 1, add, ybn, bits, aux, acc, R)
                        e.append(rel(dx3, dxa))
                        if part3.numel():
                            v = acc[: R * 2 * Cin].view(R, 2, Cin)
                            e += [rel(v[:, 0].sum(0), r_s1), rel(v[:, 1].sum(0), r_s2)]
                        acc.zero_()
                        dx4, part4 = C.conv_dgrad_bn(dy_n, wt, H, H, s, p, 1, add, ybn, bits, aux, acc, R,
                                                     ybn2, aux2)
                        e.append(rel(dx4, dxa))
                        if part4.numel():
                            v = acc.view(R, 3, Cin)
                            e += [rel(v[:, 0].sum(0), r_s1), rel(v[:, 1].sum(0), r_s2), rel(v[:, 2].sum(0), r_s3)]
                        tag = "dgrad"
                    torch.cuda.synchronize()
                finally:
                    C.conv_trial(0, -1, -1)
                if max(e) > a.tol:
                    bad.append((shape, tag, cfg, split, [round(v, 4) for v in e]))
                    print("BAD", bad[-1], flush=True)
                else:
                    n_ok += 1
        if not a.skip_wgrad:
            xg = x.detach().requires_grad_(False)
            wv = w.clone().requires_grad_(True)
            F.conv2d(xg, wv, stride=s, padding=p).backward(dy)
            ref_dw = wv.grad.permute(0, 2, 3, 1)
            for cfg, split in C.wgrad_candidates(N, H, H, Cin, Cout, k, k, s, p, 1):
                C.conv_trial(1, cfg, split)
                try:
                    dw = torch.zeros(Cout, k, k, Cin, device="cuda")
                    C.conv_wgrad(x_n, dy_n, k, k, s, p, 1, dw)
                    torch.cuda.synchronize()
                finally:
                    C.conv_trial(1, -1, -1)
                e = rel(dw, ref_dw)
                if e > a.tol:
                    bad.append((shape, "wgrad", cfg, split, round(e, 4)))
                    print("BAD", bad[-1], flush=True)
                else:
                    n_ok += 1
        print(f"{shape}: done ({n_ok} ok so far, {len(bad)} bad)", flush=True)
    print(f"SUMMARY batch {N}: {n_ok} ok, {len(bad)} bad")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
