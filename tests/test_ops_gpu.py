"""End-to-end numerics of the native GPU model path against the fp32 CPU reference path."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _compare_model(name, batch=8, tol_out=0.05, tol_grad=0.08):
    from pytorch_cifar_amd import models

    torch.manual_seed(0)
    cpu = getattr(models, name)() if not isinstance(name, tuple) else getattr(models, name[0])(*name[1:])
    gpu = copy.deepcopy(cpu).cuda()
    x = torch.randn(batch, 3, 32, 32)
    y = torch.randint(0, 10, (batch,))
    from pytorch_cifar_amd.ops.functional import cross_entropy

    out_c = cpu(x)
    loss_c = cross_entropy(out_c, y)
    loss_c.backward()
    out_g = gpu(x.cuda())
    loss_g = cross_entropy(out_g, y.cuda())
    loss_g.backward()
    torch.cuda.synchronize()
    assert rel(out_g, out_c) < tol_out, f"{name} logits rel err {rel(out_g, out_c)}"
    errs = {}
    for (n, pc), (_, pg) in zip(cpu.named_parameters(), gpu.named_parameters()):
        if pc.grad is None:
            assert pg.grad is None or pg.grad.abs().max().item() == 0, n
            continue
        errs[n] = rel(pg.grad, pc.grad)
    worst = max(errs.values())
    assert worst < tol_grad, f"{name} worst grad {max(errs, key=errs.get)} {worst}"
    for (n, bc), (_, bg) in zip(cpu.named_buffers(), gpu.named_buffers()):
        if bc.dtype.is_floating_point:
            assert rel(bg, bc) < 0.02, n
        else:
            assert int(bg.item()) == int(bc.item()), n


def test_resnet18_matches_cpu_reference():
    _compare_model("ResNet18")


def test_resnet18_trains():
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.data.loader import DeviceLoader
    from pytorch_cifar_amd.data.synthetic import synthetic_cifar10
    from pytorch_cifar_amd.engine.arena import ParamArena
    from pytorch_cifar_amd.engine.optim import SGD
    from pytorch_cifar_amd.engine.trainer import TrainStep, read_metrics

    torch.manual_seed(0)
    imgs, labs = synthetic_cifar10(512, seed=3)
    model = models.ResNet18().cuda()
    arena = ParamArena(model.parameters())
    opt = SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4).attach_arena(arena)
    loader = DeviceLoader(imgs, labs, 128, "cuda", crop_pad=4, flip=True, drop_last=True)
    step = TrainStep(model, opt, loader, 128, graph=True)
    losses = []
    for ep in range(4):
        loader.set_epoch(ep)
        for idx in loader.batch_indices():
            step(idx)
        m = read_metrics(step.metrics)
        losses.append(m[0] / len(loader))
    assert step.graph is not None, f"graph capture failed: {step.graph_error!r}"
    assert all(torch.isfinite(torch.tensor(losses))), losses
    assert losses[-1] < losses[0], losses
