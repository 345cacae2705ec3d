#!/usr/bin/env python3
"""Run ONE native conv pass on one shape repeatedly (for rocprofv3 --pmc counter collection).

  rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc -- \
      python tools/conv_one.py --cin 64 --cout 64 --h 32 --pass fwd
"""
import argparse
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
    ap.add_argument("--pass", dest="pass_", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--bn", action="store_true", help="dgrad: fused BN+ReLU backward reduce")
    ap.add_argument("--addend", action="store_true", help="dgrad: fused gradient addend")
    a = ap.parse_args()
    from pytorch_cifar_amd import _native

    C = _native.lib()
    p = a.k // 2
    Ho = (a.h + 2 * p - a.k) // a.s + 1
    x = torch.randn(a.batch, a.h, a.h, a.cin, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(a.cout, a.k, a.k, a.cin, device="cuda") * 0.05
    dy = torch.randn(a.batch, Ho, Ho, a.cout, device="cuda", dtype=torch.bfloat16)
    wb, wt = C.weight_prep(w, 1, True)
    C.set_conv_tile(0 if a.pass_ != "wgrad" else 1, a.cfg)
    add = torch.randn_like(x) if a.addend else None
    if a.bn:
        y = torch.randn_like(x)
        mask = torch.randint(0, 256, (x.numel() // 8,), device="cuda", dtype=torch.uint8)
        aux = torch.cat([torch.zeros(a.cin, device="cuda"), torch.ones(a.cin, device="cuda")])
        R = 16
        acc = torch.zeros(R * 2 * a.cin, device="cuda")

        def dgrad():
            return C.conv_dgrad_bn(dy, wt, a.h, a.h, a.s, p, 1, add, y, mask, aux, acc, R)
    else:
        def dgrad():
            return C.conv_dgrad(dy, wt, a.h, a.h, a.s, p, 1, add)
    fn = {
        "fwd": lambda: C.conv_fwd(x, wb, None, a.s, p, 1, True),
        "dgrad": dgrad,
        "wgrad": lambda: C.conv_wgrad(x, dy, a.k, a.k, a.s, p, 1, None),
    }[a.pass_]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / a.iters * 1e-3
    flops = 2.0 * a.batch * Ho * Ho * a.cout * a.cin * a.k * a.k
    tag = ("+bn" if a.bn else "") + ("+add" if a.addend else "")
    print(f"{a.pass_}{tag} {a.cin}->{a.cout} k{a.k}s{a.s}@{a.h} cfg {a.cfg}: {t * 1e6:.1f} us "
          f"{flops / t / 1e12:.0f} TF/s")


if __name__ == "__main__":
    main()
