#!/usr/bin/env python3
"""Logit / gradient error of the native path vs fp32 (CPU) next to stock bf16, per model and batch
(the tests/test_ops_gpu.py criterion, printed instead of asserted).

  python tools/debug_zoo_err.py VGG19:16 VGG19:64 VGG16:16 ...
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))

import copy  # noqa: E402

import torch  # noqa: E402

from test_ops_gpu import _grads, _run, rel  # noqa: E402


def main():
    from pytorch_cifar_amd import _native, models

    C = _native.lib()
    C.conv_autotune(False)
    C.set_deterministic(True)
    for spec in sys.argv[1:]:
        name, batch = spec.split(":")
        batch = int(batch)
        torch.manual_seed(0)
        ref = models.MODEL_REGISTRY[name]()
        nat = copy.deepcopy(ref).cuda()
        stk = copy.deepcopy(ref).cuda()
        x = torch.randn(batch, 3, 32, 32)
        y = torch.randint(0, 10, (batch,))
        o_r = _run(ref, x, y, "cpu")
        o_n = _run(nat, x, y, "cuda")
        o_s = _run(stk, x, y, "cuda", stock=True)
        gr, gn, gs = _grads(ref), _grads(nat), _grads(stk)
        worst = sorted(((rel(gn[n], g) / max(rel(gs[n], g), 1e-6), n, rel(gn[n], g), rel(gs[n], g))
                        for n, g in gr.items() if g is not None), reverse=True)[:4]
        print(f"{name} bs{batch}: logits native {rel(o_n, o_r):.4f} stock {rel(o_s, o_r):.4f}; "
              f"worst grads {[(n, round(a, 4), round(b, 4)) for _, n, a, b in worst]}", flush=True)


if __name__ == "__main__":
    main()
