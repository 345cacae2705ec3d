#!/usr/bin/env python3
"""Per-step comparison of the eager and the hipGraph TrainStep (test_graph_steps_equal_eager_steps
setup): loss after each step and the first BN's running mean, to find where they diverge."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import pytorch_cifar_amd
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.data.loader import DeviceLoader
    from pytorch_cifar_amd.data.synthetic import synthetic_cifar10
    from pytorch_cifar_amd.engine.arena import ParamArena
    from pytorch_cifar_amd.engine.optim import SGD
    from pytorch_cifar_amd.engine.trainer import TrainStep
    from pytorch_cifar_amd.ops.functional import bn_pilots

    pytorch_cifar_amd.set_deterministic(os.environ.get("DET", "1") == "1")
    imgs, labs = synthetic_cifar10(256, seed=7)
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        model = models.ResNet18().cuda()
        arena = ParamArena(model.parameters())
        opt = SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4).attach_arena(arena)
        loader = DeviceLoader(imgs, labs, 64, "cuda", crop_pad=0, flip=False, drop_last=True, seed=0)
        if os.environ.get("PRELINK") == "1" and not graph:
            # zero pilots on the convs a BN links, before the first eager step (as the graph's
            # first replay sees them): owners found on a throwaway copy's forward
            import copy

            from pytorch_cifar_amd.ops.functional import link_pilot

            probe = copy.deepcopy(model)
            with torch.no_grad():
                probe(torch.randn(64, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last))
            for n, m in probe.named_modules():
                for key, t in m.__dict__.get("_pca_pilot", {}).items():
                    link_pilot(model.get_submodule(n), t.numel(), torch.device("cuda", key))
            del probe
        step = TrainStep(model, opt, loader, 64, graph=graph)
        loader.set_epoch(0)
        rec = []
        for idx in loader.batch_indices():
            loss = step(idx)
            torch.cuda.synchronize()
            pil = bn_pilots(model)
            rec.append((float(loss), model.bn1.running_mean.clone(), arena.param_flat.clone(),
                        [p.clone() for p in pil]))
        runs.append(rec)
    for i, (a, b) in enumerate(zip(*runs)):
        dp = (a[2] - b[2]).abs().max().item()
        dr = (a[1] - b[1]).abs().max().item()
        dpil = max(((x - y).abs().max().item() for x, y in zip(a[3], b[3])), default=-1)
        print(f"step {i}: loss eager {a[0]:.6f} graph {b[0]:.6f}  d_runmean {dr:.3e}  d_param {dp:.3e}  "
              f"d_pilot {dpil:.3e}  npilot {len(a[3])}/{len(b[3])}", flush=True)


if __name__ == "__main__":
    main()
