"""The optimizer step writes the bf16 conv operands (sgd_prep_kernel, SGD.attach_weight_prep).

Oracle: the unfused pipeline — native SGD over the arena, then the WeightPrepPlan refresh at the
next forward. The fused step must give bitwise-identical masters, momenta and losses (same
arithmetic, same operands), the operands it leaves behind must equal a fresh conversion of the
masters, and a master changed behind the optimizer's back (an in-place write, a restore) must
be picked up by the next forward / graph replay.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(model_name, fused, graph, steps=4, batch=64, poke=False):
    import os

    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.data.loader import DeviceLoader
    from pytorch_cifar_amd.data.synthetic import synthetic_cifar10
    from pytorch_cifar_amd.engine.arena import ParamArena
    from pytorch_cifar_amd.engine.optim import SGD
    from pytorch_cifar_amd.engine.trainer import TrainStep

    torch.manual_seed(0)
    net = models.MODEL_REGISTRY[model_name]().cuda()
    arena = ParamArena(net.parameters())
    opt = SGD(net.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4).attach_arena(arena)
    imgs, labs = synthetic_cifar10(256, seed=1)
    loader = DeviceLoader(imgs, labs, batch, "cuda", crop_pad=0, flip=False, drop_last=True, seed=0)
    old = os.environ.get("PCA_FUSED_SGD_PREP")
    os.environ["PCA_FUSED_SGD_PREP"] = "1" if fused else "0"
    try:
        step = TrainStep(net, opt, loader, batch, graph=graph)
    finally:
        if old is None:
            del os.environ["PCA_FUSED_SGD_PREP"]
        else:
            os.environ["PCA_FUSED_SGD_PREP"] = old
    losses = []
    loader.set_epoch(0)
    for i, idx in enumerate(loader.batch_indices()):
        if i == steps:
            break
        if poke and i == 2:
            with torch.no_grad():     # a write the optimizer does not know about
                next(net.parameters()).mul_(0.5)
        losses.append(float(step(idx).detach()))
    torch.cuda.synchronize()
    if graph:
        assert step.graph is not None, step.graph_error
    plan = net.__dict__["_pca_wplan"]
    return net, arena, losses, plan


@pytest.fixture
def deterministic():
    import pytorch_cifar_amd as pca

    pca.set_deterministic(True)      # bitwise comparisons: ordered weight-gradient reductions
    yield
    pca.set_deterministic(False)


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("poke", [False, True])
def test_fused_sgd_prep_matches_unfused(deterministic, graph, poke):
    net_u, ar_u, l_u, _ = _run("ResNet18", False, graph, poke=poke)
    net_f, ar_f, l_f, plan = _run("ResNet18", True, graph, poke=poke)
    assert plan.skip_when_fresh
    assert l_f == l_u, (l_f, l_u)
    assert torch.equal(ar_f.param_flat, ar_u.param_flat)
    assert torch.equal(ar_f.mom_flat, ar_u.mom_flat)


def test_fused_sgd_operands_are_current():
    from pytorch_cifar_amd import _native
    from pytorch_cifar_amd.engine import grads as G

    net, arena, _, plan = _run("MobileNetV2", True, False, steps=3)
    C = _native.lib()
    assert plan.entries and plan.is_fresh()
    checked = 0
    for e in plan.entries:
        if isinstance(e.groups, int) and e.groups >= 1:
            wb, wt = C.weight_prep(G.physical(e.w).contiguous(), e.groups, True)
            assert torch.equal(e.wb, wb)
            assert torch.equal(e.wt, wt)
            checked += 1
        elif isinstance(e.groups, int):   # depthwise tap-major fp32 copy
            co = e.w.shape[0]
            assert torch.equal(e.wb, e.w.detach().reshape(co, -1).t().contiguous())
            checked += 1
    assert checked > 10


@pytest.mark.parametrize("name,kind", [("ShuffleNetV2_1", "gpad"), ("DPN26", "gdense")])
def test_fused_sgd_prep_padded_operands(deterministic, name, kind):
    """The fused optimizer step also writes the zero-padded operands of odd-width convs (pass 5)
    and the block-diagonal ones of narrow-group convs (pass 6): bitwise equal to the unfused
    pipeline."""
    net_u, ar_u, l_u, _ = _run(name, False, False)
    net_f, ar_f, l_f, plan = _run(name, True, False)
    assert any(isinstance(e.groups, tuple) and e.groups[0] == kind for e in plan.entries)
    assert l_f == l_u, (l_f, l_u)
    assert torch.equal(ar_f.param_flat, ar_u.param_flat)
    assert torch.equal(ar_f.mom_flat, ar_u.mom_flat)
