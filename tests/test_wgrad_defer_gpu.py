"""Deferred weight-gradient slab reductions (ops/functional.py flush_wgrads, csrc/conv_halo.hip
slab_reduce_multi_kernel): the split-K wgrads record their reduce and one batched launch runs all
of them at the end of the backward pass (or before a DDP bucket's all-reduce). Each descriptor
keeps its split-lane count and summation order, so the gradients must be bitwise those of the
per-conv reduce kernels; the fp32 oracle is covered by the zoo / production tests."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def deterministic_static():
    """Slab reductions everywhere (deterministic mode) and the static tile heuristic."""
    from pytorch_cifar_amd import _native

    C = _native.lib()
    det, at = C.deterministic(), C.conv_autotune_enabled()
    C.set_deterministic(True)
    C.conv_autotune(False)
    yield C
    C.set_deterministic(det)
    C.conv_autotune(at)


def _grads(model, x, y, defer, monkeypatch, counts):
    from pytorch_cifar_amd.engine.arena import ParamArena
    from pytorch_cifar_amd.ops import functional as F

    if defer == "piggy":
        monkeypatch.setattr(F, "_WGRAD_DEFER", False)
        monkeypatch.setattr(F, "_WGRAD_PIGGY", True)
    else:
        monkeypatch.setattr(F, "_WGRAD_DEFER", defer)
        monkeypatch.setattr(F, "_WGRAD_PIGGY", False)
    flush = F.flush_wgrads

    def counting_flush():
        counts.append(F._C().wgrad_deferred())
        flush()

    monkeypatch.setattr(F, "flush_wgrads", counting_flush)
    arena = ParamArena(list(model.parameters()))
    out = model(x)
    F.cross_entropy(out, y).backward()
    torch.cuda.synchronize()
    assert F._C().wgrad_deferred() == 0, "a deferred reduction was left pending after backward"
    g = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    del arena
    return g


@pytest.mark.parametrize("name,batch", [("ResNet18", 128), ("ResNet18", 32), ("ResNet50", 16)])
def test_deferred_wgrad_reduce_bitwise(name, batch, monkeypatch, deterministic_static):
    from pytorch_cifar_amd import models

    torch.manual_seed(0)
    m0 = models.MODEL_REGISTRY[name]().cuda()
    m1 = copy.deepcopy(m0)
    x = torch.randn(batch, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (batch,), device="cuda")
    on, off = [], []
    ga = _grads(m0, x, y, True, monkeypatch, on)
    gb = _grads(m1, x, y, False, monkeypatch, off)
    assert sum(on) > 0, "no weight gradient took the deferred path"
    assert sum(off) == 0
    bad = [n for n in ga if not torch.equal(ga[n], gb[n])]
    assert not bad, f"deferred reduce differs: {bad[:8]}"


def test_flush_outside_backward_is_immediate(deterministic_static):
    """A deferred wgrad issued outside an autograd pass is flushed at once (nobody else would)."""
    from pytorch_cifar_amd.ops import functional as F

    C = deterministic_static
    x = torch.randn(64, 16, 16, 64, device="cuda").to(torch.bfloat16)
    dy = torch.randn(64, 16, 16, 64, device="cuda").to(torch.bfloat16)
    ref = C.conv_wgrad(x, dy, 3, 3, 1, 1, 1, torch.zeros(64, 3, 3, 64, device="cuda"))
    buf = torch.zeros(64, 3, 3, 64, device="cuda")
    C.conv_wgrad(x, dy, 3, 3, 1, 1, 1, buf, defer=True)
    if C.wgrad_deferred():
        F._after_deferred_wgrad()
    assert C.wgrad_deferred() == 0
    torch.cuda.synchronize()
    assert torch.equal(buf, ref)


def test_piggyback_reduce_unit(deterministic_static):
    """A recorded slab reduction rides along in the next fused BatchNorm-backward launch
    (csrc/batchnorm.hip bn_bwd_apply_acc_rows_red_kernel): nothing left pending, the weight
    gradient equal to the per-conv reduce kernel's up to fp32 summation order, and the BN pass
    itself bitwise the launch without passengers."""
    C = deterministic_static
    torch.manual_seed(1)
    N, H, Cc = 32, 16, 64
    x = torch.randn(N, H, H, Cc, device="cuda").to(torch.bfloat16)
    dyw = torch.randn(N, H, H, Cc, device="cuda").to(torch.bfloat16)
    ref = C.conv_wgrad(x, dyw, 3, 3, 1, 1, 1, torch.zeros(Cc, 3, 3, Cc, device="cuda"))
    # a fused BN backward (accumulator form, sums already delivered)
    M = N * H * H
    y = torch.randn(N, H, H, Cc, device="cuda").to(torch.bfloat16)
    dout = torch.randn(N, H, H, Cc, device="cuda").to(torch.bfloat16)
    mask = torch.randint(0, 256, (M * Cc // 8,), device="cuda", dtype=torch.uint8)
    aux = torch.cat([torch.randn(Cc, device="cuda") * 0.1, torch.rand(Cc, device="cuda") + 0.5,
                     torch.rand(Cc, device="cuda"), torch.randn(Cc, device="cuda")])
    gamma = torch.rand(Cc, device="cuda") + 0.5
    R = 4
    sums = torch.randn(R * 2 * Cc, device="cuda")

    def bwd():
        acc = sums.clone()
        return C.bn_backward(dout, None, mask, y, aux, gamma, None, None, None, 1, True, False,
                             None, None, None, None, None, acc, R, True, None, None, None, False,
                             None)[0]

    base = bwd()
    C.wgrad_piggy(True)
    try:
        buf = torch.zeros(Cc, 3, 3, Cc, device="cuda")
        C.conv_wgrad(x, dyw, 3, 3, 1, 1, 1, buf, defer=True)
        assert C.wgrad_deferred() == 1, "the slab wgrad did not record its reduction"
        got = bwd()
        assert C.wgrad_deferred() == 0, "the BN launch did not take the pending reduction"
    finally:
        C.wgrad_piggy(False)
    torch.cuda.synchronize()
    assert torch.equal(got, base)
    d = (buf - ref).abs().max().item()
    assert d <= 1e-5 * ref.abs().max().item(), d


@pytest.mark.parametrize("name,batch", [("ResNet18", 128), ("ResNet18", 1024)])
def test_piggyback_wgrad_reduce_model(name, batch, monkeypatch):
    """Production mode (autotuned selections, sharded BN accumulators): the split-K wgrads'
    reductions are taken by the BN-backward launches (at most a few left for the end-of-pass
    flush) and the gradients agree with the per-conv reduce launches to bf16 tolerance."""
    from pytorch_cifar_amd import models

    torch.manual_seed(0)
    m0 = models.MODEL_REGISTRY[name]().cuda()
    m1 = copy.deepcopy(m0)
    x = torch.randn(batch, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (batch,), device="cuda")
    left = []
    ga = _grads(m0, x, y, "piggy", monkeypatch, left)
    gb = _grads(m1, x, y, False, monkeypatch, [])
    for n in ga:
        d = (ga[n] - gb[n]).abs().max().item()
        s = gb[n].abs().max().item()
        assert d <= 2e-2 * max(s, 1e-12), (n, d, s)
    assert sum(left) <= 3, f"{sum(left)} reductions left for the end-of-pass flush"
