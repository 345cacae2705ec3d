"""Model-zoo parity with the reference (CPU, fp32).

For every constructor: identical state_dict keys and shapes as the reference model, the
reference's weights load strictly, and forward (eval and train mode) plus input/parameter
gradients match the reference implementation. The reference package is imported read-only from
/root/reference when present (skipped elsewhere, e.g. on the GPU box). ShuffleNetG2/G3 cannot be
constructed by the reference under Python 3 (shufflenet.py:27 float channels) — our fixed
version is checked for shape/contract only.
"""
import copy
import importlib.util
import os
import sys

import pytest
import torch

REF = "/root/reference/models/__init__.py"

ZOO = [
    "VGG11", "VGG13", "VGG16", "VGG19", "LeNet", "ResNet18", "ResNet34", "ResNet50",
    "PreActResNet18", "PreActResNet50", "GoogLeNet", "DenseNet121", "densenet_cifar",
    "ResNeXt29_2x64d", "ResNeXt29_32x4d", "MobileNet", "MobileNetV2", "DPN26", "SENet18",
    "EfficientNetB0", "RegNetX_200MF", "RegNetX_400MF", "RegNetY_400MF", "SimpleDLA", "DLA",
    "PNASNetA", "PNASNetB", "ShuffleNetV2_0.5", "ShuffleNetV2_1",
]
HEAVY = ["ResNet101", "ResNet152", "PreActResNet34", "PreActResNet101", "PreActResNet152",
         "DenseNet169", "DenseNet201", "DenseNet161", "ResNeXt29_4x64d", "ResNeXt29_8x64d",
         "DPN92", "ShuffleNetV2_1.5", "ShuffleNetV2_2"]


@pytest.fixture(scope="module")
def ref_models():
    if not os.path.exists(REF):
        pytest.skip("reference checkout not available")
    spec = importlib.util.spec_from_file_location(
        "pca_reference_models", REF, submodule_search_locations=[os.path.dirname(REF)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["pca_reference_models"] = mod
    spec.loader.exec_module(mod)
    return mod


def _ref_ctor(ref, name):
    if name.startswith("VGG"):
        return lambda: ref.VGG(name)
    if name.startswith("ShuffleNetV2_"):
        s = float(name.split("_")[1])
        s = int(s) if s.is_integer() else s
        return lambda: ref.ShuffleNetV2(s)
    return getattr(ref, name)


def _ours(name):
    from pytorch_cifar_amd import models

    return models.MODEL_REGISTRY[name]()


def _rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


def _run(model, x, g, seed):
    xi = x.clone().requires_grad_(True)
    torch.manual_seed(seed)
    y = model(xi)
    y.backward(g.to(y.dtype))
    grads = {n: p.grad for n, p in model.named_parameters()}
    return y.detach(), xi.grad, grads


def _check(name, ref):
    """fp64 run of the reference model is the oracle; our fp32 model must be as close to it as
    the reference's own fp32 run is (BN backward at batch 4 is ill-conditioned in fp32, so the
    two fp32 runs legitimately differ by ~1e-3 in the input gradient while agreeing to 1e-15 in
    fp64 — checked separately by test_zoo_exact_in_fp64)."""
    torch.manual_seed(0)
    r = _ref_ctor(ref, name)()
    o = _ours(name)
    rs, os_ = r.state_dict(), o.state_dict()
    assert list(rs.keys()) == list(os_.keys()), name
    for k in rs:
        assert rs[k].shape == os_[k].shape, (name, k)
    o.load_state_dict(rs, strict=True)
    r64 = copy.deepcopy(r).double()
    x = torch.randn(4, 3, 32, 32)
    r.eval(), o.eval(), r64.eval()
    with torch.no_grad():
        oracle = r64(x.double())
        assert _rel(o(x), oracle) <= 3 * _rel(r(x), oracle) + 1e-6, f"{name} eval logits"
    r.train(), o.train(), r64.train()
    g = torch.randn(4, 10)
    y64, gx64, gp64 = _run(r64, x.double(), g, 1)
    yr, gxr, gpr = _run(r, x, g, 1)
    yo, gxo, gpo = _run(o, x, g, 1)
    assert _rel(yo, y64) <= 3 * _rel(yr, y64) + 1e-6, f"{name} train logits"
    assert _rel(gxo, gx64) <= 3 * _rel(gxr, gx64) + 1e-6, f"{name} input grad"
    for n, g64 in gp64.items():
        if g64 is None:
            assert gpo[n] is None or gpo[n].abs().max() == 0, n
            continue
        assert _rel(gpo[n], g64) <= 3 * _rel(gpr[n], g64) + 1e-6, f"{name}.{n}"
    for (n, br), (_, bo) in zip(r.named_buffers(), o.named_buffers()):
        if br.dtype.is_floating_point:
            assert _rel(bo, br) < 1e-4 or (bo - br).abs().max() < 1e-6, f"{name}.{n}"
        else:
            assert int(bo) == int(br), f"{name}.{n}"


@pytest.mark.parametrize("name", ZOO)
def test_zoo_matches_reference(ref_models, name):
    _check(name, ref_models)


@pytest.mark.slow
@pytest.mark.parametrize("name", HEAVY)
def test_heavy_zoo_matches_reference(ref_models, name):
    _check(name, ref_models)


def test_registry_complete():
    from pytorch_cifar_amd import models

    assert len(models.MODEL_REGISTRY) == 44
    for name in ["VGG", "LeNet", "ResNet18", "ResNet152", "PreActResNet152", "GoogLeNet", "DenseNet161",
                 "densenet_cifar", "ResNeXt29_32x4d", "MobileNet", "MobileNetV2", "DPN92",
                 "ShuffleNetG2", "ShuffleNetG3", "ShuffleNetV2", "SENet18", "EfficientNetB0",
                 "RegNetX_200MF", "RegNetX_400MF", "RegNetY_400MF", "SimpleDLA", "DLA",
                 "PNASNetA", "PNASNetB"]:
        assert hasattr(models, name), name


@pytest.mark.parametrize("name", ["ShuffleNetG2", "ShuffleNetG3"])
def test_shufflenet_g_fixed(name):
    m = _ours(name)
    y = m(torch.randn(2, 3, 32, 32))
    assert y.shape == (2, 10)
    y.sum().backward()


def test_resnet_amp_flag_accepted():
    from pytorch_cifar_amd import models

    m = models.ResNet18(amp=True)
    assert m.amp and m.layer1[0].amp


@pytest.mark.parametrize("name", ["ResNet18", "EfficientNetB0", "DLA", "ShuffleNetV2_1", "DPN26"])
def test_zoo_exact_in_fp64(ref_models, name):
    torch.manual_seed(0)
    r = _ref_ctor(ref_models, name)().double()
    o = _ours(name).double()
    o.load_state_dict(r.state_dict())
    x = torch.randn(3, 3, 32, 32, dtype=torch.float64)
    g = torch.randn(3, 10, dtype=torch.float64)
    yr, gxr, gpr = _run(r, x, g, 2)
    yo, gxo, gpo = _run(o, x, g, 2)
    assert _rel(yo, yr) < 1e-12 and _rel(gxo, gxr) < 1e-10
    for n, gr in gpr.items():
        if gr is not None and gr.norm() > 1e-8:
            assert _rel(gpo[n], gr) < 1e-9, n
