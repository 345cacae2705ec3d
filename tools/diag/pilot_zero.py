#!/usr/bin/env python3
"""One training step (forward + backward; GRAD=0: forward only) of ResNet-18 twice from identical weights: (a) a fresh model (the convs have
no BN pilot yet: unshifted sums), (b) a copy whose convs already hold zero pilots (shift K = 0).
The two must agree bitwise; prints the first module output / parameter gradient that differs."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import pytorch_cifar_amd
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.ops.functional import link_pilot

    pytorch_cifar_amd.set_deterministic(os.environ.get("DET", "1") == "1")
    torch.manual_seed(0)
    bs = int(os.environ.get("BS", "64"))
    base = models.ResNet18().cuda().train()
    x = torch.randn(bs, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    labels = torch.randint(0, 10, (bs,), device="cuda")

    def run(model):
        outs = []
        hooks = [m.register_forward_hook(lambda m, i, o, n=n: outs.append((n, o.detach().float().clone())))
                 for n, m in model.named_modules() if n]
        if os.environ.get("GRAD", "1") == "1":
            from pytorch_cifar_amd.ops.functional import cross_entropy

            y = model(x)
            loss = cross_entropy(y, labels)
            loss.backward()
        else:
            with torch.no_grad():
                y = model(x)
        torch.cuda.synchronize()
        for h in hooks:
            h.remove()
        grads = [(n, p.grad.float().clone()) for n, p in model.named_parameters() if p.grad is not None]
        return y.float(), outs + grads

    a = copy.deepcopy(base)
    ya, oa = run(a)
    # the convs that got a pilot in (a) get a zero one in (b) before its first forward
    b = copy.deepcopy(base)
    owners = {n for n, m in a.named_modules() if m.__dict__.get("_pca_pilot")}
    for n, m in b.named_modules():
        if n in owners:
            for key, t in dict(a.get_submodule(n).__dict__["_pca_pilot"]).items():
                link_pilot(m, t.numel(), torch.device("cuda", key))
    yb, ob = run(b)
    print(f"pilots: {len(owners)}; logits equal: {torch.equal(ya, yb)}  max diff {(ya - yb).abs().max().item():.3e}")
    for (na, ta), (nb, tb) in zip(oa, ob):
        if not torch.equal(ta, tb):
            print(f"first difference: {na} ({nb}) max {(ta - tb).abs().max().item():.3e} shape {tuple(ta.shape)}")
            break
    else:
        print("all module outputs bitwise equal")


if __name__ == "__main__":
    main()
