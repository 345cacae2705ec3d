"""End-to-end numerics of the native GPU model path.

Oracle: the same model (same weights) run in fp32 on the CPU reference path. Because the GPU
path computes in bf16, its error against the oracle is compared with the error of the *stock*
bf16 path — the identical model run on the GPU through stock PyTorch kernels under
``torch.autocast(bfloat16)`` (``reference_kernels()`` mode). The native path must be as close
to fp32 as stock bf16 PyTorch is (within a small factor), for logits and every gradient.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _grads(model):
    return {n: p.grad for n, p in model.named_parameters()}


def _run(model, x, y, device, stock=False):
    from pytorch_cifar_amd.ops.functional import cross_entropy, reference_kernels

    x, y = x.to(device), y.to(device)
    if stock:
        with reference_kernels(), torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(x.contiguous(memory_format=torch.channels_last))
            loss = cross_entropy(out.float(), y)
        loss.backward()
    else:
        out = model(x)
        loss = cross_entropy(out, y)
        loss.backward()
    torch.cuda.synchronize() if device == "cuda" else None
    return out.float()


def compare_model(ctor, batch=32, factor=3.0, slack=0.01, check_buffers=True, warm=0,
                  return_models=False):
    torch.manual_seed(0)
    ref = ctor()
    native = copy.deepcopy(ref).cuda()
    stock = copy.deepcopy(ref).cuda()
    for _ in range(warm):
        # earlier training steps (running stats move, the convs switch their BN statistics to
        # the sharded accumulators once a BN consumed them): compare the step after
        xw = torch.randn(batch, 3, 32, 32)
        yw = torch.randint(0, 10, (batch,))
        _run(ref, xw, yw, "cpu")
        _run(native, xw, yw, "cuda")
        _run(stock, xw, yw, "cuda", stock=True)
        for m in (ref, native, stock):
            for p in m.parameters():
                p.grad = None
    x = torch.randn(batch, 3, 32, 32)
    y = torch.randint(0, 10, (batch,))
    out_r = _run(ref, x, y, "cpu")
    out_n = _run(native, x, y, "cuda")
    out_s = _run(stock, x, y, "cuda", stock=True)
    e_n, e_s = rel(out_n, out_r), rel(out_s, out_r)
    assert e_n <= factor * e_s + slack, f"logits: native {e_n:.4f} vs stock-bf16 {e_s:.4f}"
    gr, gn, gs = _grads(ref), _grads(native), _grads(stock)
    # a parameter whose fp32 gradient is numerically zero (norm < 1e-6 x the median gradient
    # norm: e.g. a bias feeding a training-mode BatchNorm) has no meaningful relative error
    norms = sorted(g.norm().item() for g in gr.values() if g is not None)
    scale = norms[len(norms) // 2] if norms else 0.0
    # relative-error floor: the squeeze-excite MLP gradients (SENet / RegNetY / EfficientNet)
    # are sums over the image that nearly cancel at init, so BOTH bf16 paths land at 0.05-0.5
    # relative error on them and which of the two is lower at one seed is chance (measured over
    # seeds with tools/debug_senet.py). A parameter's stock error is therefore floored at the
    # median stock error of the parameters of its kind (SE MLP vs the rest).
    errs = {n: (rel(gn[n], g), rel(gs[n], g)) for n, g in gr.items() if g is not None}

    def _se(n):
        return ".fc1." in n or ".fc2." in n or ".se." in n

    def _median(vals):
        vals = sorted(vals)
        return vals[len(vals) // 2] if vals else 0.0

    floor = {k: _median([e[1] for n, e in errs.items() if _se(n) == k]) for k in (True, False)}
    bad = []
    for name, g in gr.items():
        if g is None:
            assert gn[name] is None or gn[name].abs().max().item() == 0, name
            continue
        en, es = errs[name]
        es = max(es, floor[_se(name)]) if _se(name) else es
        small = g.norm().item() < 1e-6 * scale
        if en > factor * es + slack and not small:
            bad.append((name, round(en, 4), round(es, 4)))
    assert not bad, f"grads worse than stock bf16 (name, native, stock): {bad[:10]}"
    if check_buffers:
        bufs_s = dict(stock.named_buffers())
        for (n, br), (_, bn) in zip(ref.named_buffers(), native.named_buffers()):
            if br.dtype.is_floating_point:
                # running stats: same criterion as the gradients, or absolutely negligible (a BN
                # fed by a zero-mean producer has running_mean ~1e-9 in fp32, ~1e-6 in bf16)
                en, es = rel(bn, br), rel(bufs_s[n], br)
                small = (bn.float().cpu() - br.float()).abs().max().item() < 1e-4
                assert en <= factor * es + slack or small, (n, en, es)
            else:
                assert int(bn.item()) == int(br.item()), n
    if return_models:
        return e_n, e_s, native
    return e_n, e_s


def test_resnet18_matches_reference():
    from pytorch_cifar_amd import models

    compare_model(models.ResNet18)


def test_resnet18_trains():
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.data.loader import DeviceLoader
    from pytorch_cifar_amd.data.synthetic import synthetic_cifar10
    from pytorch_cifar_amd.engine.arena import ParamArena
    from pytorch_cifar_amd.engine.optim import SGD
    from pytorch_cifar_amd.engine.trainer import TrainStep, read_metrics

    torch.manual_seed(0)
    # no augmentation: the 256 images are memorised within a few epochs (CPU fp32 run of the same
    # recipe: 2.39 -> 1.51 -> 0.52 -> 0.04), so a working step must drive the loss well down
    imgs, labs = synthetic_cifar10(256, seed=3)
    model = models.ResNet18().cuda()
    arena = ParamArena(model.parameters())
    opt = SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4).attach_arena(arena)
    loader = DeviceLoader(imgs, labs, 128, "cuda", crop_pad=0, flip=False, drop_last=True)
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
    assert losses[-1] < 0.5 * losses[0], losses


GPU_ZOO = ["LeNet", "VGG11", "PreActResNet18", "GoogLeNet", "densenet_cifar", "ResNeXt29_2x64d",
           "MobileNet", "MobileNetV2", "DPN26", "SENet18", "EfficientNetB0", "RegNetX_200MF",
           "RegNetY_400MF", "SimpleDLA", "DLA", "PNASNetA", "PNASNetB", "ShuffleNetG2",
           "ShuffleNetV2_1", "ResNet50", "ResNeXt29_32x4d",
           # the reference's documented workload (main_dist.py:136, train.sh) and the deep / wide
           # variants: DenseNet161's dense3 / dense4 (2112 / 2208 channels) exceed the row-tiled BN
           # kernels' 2048 and must take the copying concat there
           "ResNet152", "PreActResNet152", "DenseNet121", "DenseNet161", "DenseNet201", "DPN92",
           "ResNeXt29_8x64d", "VGG19"]


@pytest.fixture
def reproducible_convs():
    """Static tile heuristic + deterministic reductions: the timing-based autotuner may pick a
    different (equally valid, separately tested) tile/split per run, which moves bf16 rounding
    around; near-cancelling gradients (SE biases) then pass or fail by chance."""
    from pytorch_cifar_amd import _native

    C = _native.lib()
    at, det = C.conv_autotune_enabled(), C.deterministic()
    C.conv_autotune(False)
    C.conv_clear_tuned()         # choices tuned by earlier tests would override the heuristic
    C.set_deterministic(True)
    yield
    C.conv_autotune(at)
    C.set_deterministic(det)


@pytest.mark.parametrize("name", GPU_ZOO)
def test_zoo_matches_reference(name, reproducible_convs):
    """Every model family through the native kernels: as close to fp32 as stock bf16."""
    from pytorch_cifar_amd import models

    def ctor():
        m = models.MODEL_REGISTRY[name]()
        if hasattr(m, "cfg") and isinstance(m.cfg, dict) and "dropout_rate" in m.cfg:
            m.cfg = dict(m.cfg, dropout_rate=0.0)  # CPU and GPU dropout masks differ
        return m

    compare_model(ctor, batch=16)


@pytest.fixture
def static_tiles():
    """Static conv tile heuristic (no timing-based autotune), non-deterministic mode (the sharded
    BN accumulators are on)."""
    from pytorch_cifar_amd import _native

    C = _native.lib()
    at, det = C.conv_autotune_enabled(), C.deterministic()
    C.conv_autotune(False)
    C.set_deterministic(False)
    yield
    C.conv_autotune(at)
    C.set_deterministic(det)


@pytest.mark.parametrize("name", ["ResNet18", "ResNet50", "PreActResNet18", "MobileNetV2",
                                  "EfficientNetB0", "RegNetY_400MF", "densenet_cifar", "DLA",
                                  "SENet18", "DenseNet121"])
def test_bn_accumulators_match_reference(name, static_tiles):
    """Steps after the first route every conv->BN statistic and every BN-backward sum through the
    sharded accumulators (fused finalize in the BN kernels; DenseNet121: the dense slabs'
    statistics cache and the suffix BNs' backward sums from row-strided dgrad epilogues): still
    as close to fp32 as stock bf16, running stats / num_batches_tracked exact in count, and after the step every forward
    accumulator is back at zero (cleared by its BN's backward kernel); the backward ones are
    cleared by the next forward."""
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.ops.functional import StatAcc

    def ctor():
        m = models.MODEL_REGISTRY[name]()
        if hasattr(m, "cfg") and isinstance(m.cfg, dict) and "dropout_rate" in m.cfg:
            m.cfg = dict(m.cfg, dropout_rate=0.0)
        return m

    _, _, native = compare_model(ctor, batch=16, warm=2, return_models=True)
    items = [(k, a) for mod in native.modules() for k, a in mod.__dict__.get("_pca_acc", {}).items()]
    assert items, "no module switched to accumulator statistics"
    torch.cuda.synchronize()
    for k, a in items:
        assert isinstance(a, StatAcc)
        if k[0] in ("fwd", "fwdstat"):
            assert a.state == "clean", (k, a.state)
        if a.state == "clean":
            assert a.buf.abs().max().item() == 0, f"{k}: accumulator marked clean is not zero"
    with torch.no_grad():
        native(torch.randn(16, 3, 32, 32, device="cuda"))
    torch.cuda.synchronize()
    for k, a in items:
        if k[0] == "bwd":
            assert a.state == "clean" and a.buf.abs().max().item() == 0, k
    if name == "ResNet18":
        fwd = [a for k, a in items if k[0] == "fwd"]
        bwd = [a for k, a in items if k[0] == "bwd"]
        # 20 BNs: every conv feeds one; the 3 projection-shortcut BNs are folded into their
        # block's second BN kernel (dual BN), which owns the shared backward accumulator
        assert len(fwd) >= 19 and len(bwd) >= 17, (len(fwd), len(bwd))


@pytest.mark.parametrize("name", ["ResNet18", "MobileNetV2"])
def test_batched_weight_prep_matches_per_conv(name, reproducible_convs):
    """The one-launch weight conversion (forward pre-hook; MFMA conv operands and the depthwise
    tap-major copies) produces the same forward/backward as per-conv conversion, and follows
    in-place weight updates (it re-converts every forward).
    Deterministic mode: with fp32-atomic BatchNorm sums the backward chain of two identical
    models differs in bf16 rounding, so it would not isolate the weight conversion."""
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.engine.arena import ParamArena
    from pytorch_cifar_amd.ops.functional import DW_PREP, cross_entropy, enable_batched_weight_prep

    torch.manual_seed(0)
    a = models.MODEL_REGISTRY[name]().cuda()
    b = copy.deepcopy(a)
    ParamArena(a.parameters())
    ParamArena(b.parameters())
    enable_batched_weight_prep(b)
    x = torch.randn(16, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (16,), device="cuda")
    convs = [n for n, m in a.named_modules()
             if isinstance(getattr(m, "weight", None), torch.Tensor) and m.weight.dim() == 4]
    dw = [n for n, m in a.named_modules() if getattr(m, "groups", 1) > 1]
    for it in range(2):
        outs = []
        for m in (a, b):
            for p in m.parameters():
                p.grad.zero_()
            out = m(x)
            cross_entropy(out, y).backward()
            outs.append(out.float())
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1]), it
        ga = dict(a.named_parameters())
        for n, p in b.named_parameters():
            torch.testing.assert_close(p.grad, ga[n].grad, rtol=1e-2, atol=1e-4)
        with torch.no_grad():   # an in-place update that does not go through the optimizer
            for m in (a, b):
                mods = dict(m.named_modules())
                mods[convs[0]].weight.mul_(0.5)
                mods[convs[5]].weight.add_(0.01)
                if dw:
                    mods[dw[1]].weight.mul_(-0.7)
    entries = b.__dict__["_pca_wplan"].entries
    assert len(entries) >= 19
    if dw:
        assert sum(e.groups == DW_PREP for e in entries) >= len(dw) - 1


def test_bn_backward_reduce_fusion_matches_separate_pass():
    """BN+ReLU backward with its (sum dz, sum dz*xhat) reduced in the consumer conv's dgrad
    epilogue (igemm, split-K reduce and layer-1 c64 kernels) equals the separate-pass reduce."""
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.ops import functional as PF

    torch.manual_seed(0)
    base = models.ResNet18().cuda()
    x = torch.randn(64, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (64,), device="cuda")
    grads = []
    try:
        for fuse in (False, True):
            PF.set_fuse_bn_backward(fuse)
            m = copy.deepcopy(base)
            PF.cross_entropy(m(x), y).backward()
            torch.cuda.synchronize()
            grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    finally:
        PF.set_fuse_bn_backward(True)
    bad = []
    for n, g0 in grads[0].items():
        e = rel(grads[1][n], g0)
        if e > 2e-2:
            bad.append((n, round(e, 4)))
    assert not bad, bad


@pytest.mark.parametrize("N,H,C", [(16, 4, 512), (128, 4, 512), (64, 16, 128), (32, 8, 256)])
def test_conv_dgrad_dual_bn_sums(N, H, C):
    """conv_dgrad_bn with a dual-BN request: dX and the three accumulator sums (dz, dz*xhat,
    dz*xhat2 with dz = dX * mask) against torch on the same bf16 dX."""
    from pytorch_cifar_amd import _native
    from pytorch_cifar_amd.ops import functional as PF

    Cn = _native.lib()
    torch.manual_seed(23)
    dy = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = torch.randn(C, C, 3, 3, device="cuda") * 0.05
    wb, wt = Cn.weight_prep(w.permute(0, 2, 3, 1).contiguous(), 1, True)
    y = torch.randn(N, H, H, C, device="cuda").bfloat16()
    y2 = (torch.randn(N, H, H, C, device="cuda") * 2 + 0.5).bfloat16()
    mask_bits = torch.rand(N * H * H * C, device="cuda") > 0.4
    mask = (mask_bits.view(-1, 8).to(torch.uint8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1).to(torch.uint8)
    aux = torch.cat([torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5,
                     torch.zeros(2 * C, device="cuda")])
    aux2 = torch.cat([torch.randn(C, device="cuda") * 0.3 + 0.5, torch.rand(C, device="cuda") + 0.5,
                      torch.zeros(2 * C, device="cuda")])
    R = PF.acc_shards(C)
    acc = torch.zeros(R * 3 * C, device="cuda")
    dx, part = Cn.conv_dgrad_bn(dy, wt, H, H, 1, 1, 1, None, y, mask, aux, acc, R, y2, aux2)
    ref = torch.nn.functional.conv_transpose2d(dy.permute(0, 3, 1, 2).float(), w, padding=1)
    assert rel(dx.permute(0, 3, 1, 2).float(), ref) < 1e-2
    if part.numel() == 0:
        pytest.skip("selected dgrad kernel cannot fuse a dual BN")
    dz = dx.float().reshape(-1, C) * mask_bits.view(-1, C).float()
    xh = (y.float().reshape(-1, C) - aux[:C]) * aux[C:2 * C]
    xh2 = (y2.float().reshape(-1, C) - aux2[:C]) * aux2[C:2 * C]
    got = acc.view(R, 3, C).sum(0)
    assert rel(got[0], dz.sum(0)) < 1e-3
    assert rel(got[1], (dz * xh).sum(0)) < 1e-3
    assert rel(got[2], (dz * xh2).sum(0)) < 1e-3


@pytest.mark.parametrize("batch", [128, 256])
def test_dual_bn_backward_reduce_fusion(batch):
    """Projection-shortcut block tails act(BN(y) + BN2(y2)): the three backward sums reduced in
    the consumer conv's dgrad epilogue (igemm) or split-K reduce equal the separate reduce pass —
    every parameter gradient after one step (a second step is not comparable: fp32-atomic BN sums
    make its forward differ at bf16-rounding level, amplified through 20 layers)."""
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.ops import functional as PF

    torch.manual_seed(3)
    base = models.ResNet18().cuda()
    x = torch.randn(batch, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (batch,), device="cuda")
    grads = []
    try:
        for fuse in (False, True):
            PF.set_dual_bn_fuse(fuse)
            m = copy.deepcopy(base)
            PF.cross_entropy(m(x), y).backward()
            torch.cuda.synchronize()
            grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters()})
    finally:
        PF.set_dual_bn_fuse(True)
    bad = []
    for n, g0 in grads[0].items():
        e = rel(grads[1][n], g0)
        if e > 2e-2:
            bad.append((n, round(e, 4)))
    assert not bad, bad


@pytest.mark.parametrize("mode", ["1", "0", "all"])
@pytest.mark.parametrize("Cin,Cout,G,k,s", [(200, 50, 2, 1, 1), (50, 176, 2, 1, 1), (96, 96, 32, 3, 2),
                                           (128, 128, 32, 3, 1), (12, 44, 1, 3, 1), (3, 6, 1, 5, 1),
                                           (192, 192, 8, 3, 1), (96, 96, 32, 3, 1)])
def test_group_padded_conv_matches_fp32(Cin, Cout, G, k, s, mode, monkeypatch):
    """Narrow groups on the MFMA GEMM — as block-diagonal super-groups (PCA_GROUP_DENSE 1 / all)
    or zero-padded to multiples of 8 (0): output, BN statistics, dX, dW against fp32 F.conv2d."""
    import torch.nn.functional as F
    from pytorch_cifar_amd.ops import functional as OF

    monkeypatch.setattr(OF, "_GROUP_DENSE", mode)

    torch.manual_seed(7)
    p = k // 2
    x = torch.randn(4, Cin, 12, 12, device="cuda").bfloat16().float().requires_grad_(True)
    w = (torch.randn(Cout, Cin // G, k, k, device="cuda") * 0.2).requires_grad_(True)
    wn = w.detach().clone().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    ref = F.conv2d(x, w, None, s, p, 1, G)
    y, stats = OF.conv2d(x.detach().requires_grad_(True), wn, None, s, p, G, True)
    assert rel(y, ref) < 1e-2
    st = stats.sum(0)
    assert rel(st[0], ref.detach().sum((0, 2, 3))) < 2e-2
    assert rel(st[1], (ref.detach() ** 2).sum((0, 2, 3))) < 2e-2
    dy = torch.randn_like(ref).bfloat16().float()
    ref.backward(dy)
    # activations reach a conv as bf16 NHWC storage (fp32 NCHW input is the image-conversion path)
    xn = x.detach().bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y, _ = OF.conv2d(xn, wn, None, s, p, G, False)
    y.backward(dy.to(y.dtype))
    assert rel(xn.grad, x.grad) < 2e-2
    assert rel(wn.grad, w.grad) < 2e-2


@pytest.mark.parametrize("Cin,Cout,G", [(200, 50, 2), (12, 44, 1), (96, 75, 3)])
def test_group_padded_conv_bias_and_native_remaps(Cin, Cout, G):
    """The padded grouped conv's pad / slice are native remaps (no stock pad / slice kernels):
    a biased conv's output, dX, dW, db vs fp32, with dW / db added into existing gradients."""
    import torch.nn.functional as F
    from pytorch_cifar_amd.ops import functional as OF

    torch.manual_seed(17)
    x = torch.randn(3, Cin, 9, 9, device="cuda").bfloat16().float().requires_grad_(True)
    w = (torch.randn(Cout, Cin // G, 3, 3, device="cuda") * 0.2).requires_grad_(True)
    b = torch.randn(Cout, device="cuda").requires_grad_(True)
    ref = F.conv2d(x, w, b, 1, 1, 1, G)
    dy = torch.randn_like(ref).bfloat16().float()
    ref.backward(dy)
    wn = w.detach().clone().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    bn = b.detach().clone().requires_grad_(True)
    wn.grad = torch.ones_like(wn)            # accumulation into an existing gradient buffer
    bn.grad = torch.ones_like(bn)
    xn = x.detach().bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    with torch.autograd.profiler.profile(use_device="cuda") as prof:
        y, _ = OF.conv2d(xn, wn, bn, 1, 1, G, False)
        y.backward(dy.to(y.dtype).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
    assert rel(y, ref) < 1e-2
    assert rel(xn.grad, x.grad) < 2e-2
    assert rel(wn.grad - 1, w.grad) < 2e-2
    assert rel(bn.grad - 1, b.grad) < 2e-2
    names = " ".join(e.name for e in prof.function_events)
    assert "constant_pad" not in names and "aten::slice_backward" not in names, names


@pytest.mark.parametrize("C,g", [(200, 2), (240, 3), (64, 4), (30, 3)])
def test_channel_shuffle_native(C, g):
    """ShuffleNet channel shuffle as a native remap (fwd + bwd) vs the reshape/transpose oracle."""
    from pytorch_cifar_amd.ops import functional as OF

    torch.manual_seed(18)
    x = torch.randn(2, C, 5, 7, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xr = x.float().requires_grad_(True)
    ref = xr.reshape(2, g, C // g, 5, 7).transpose(1, 2).reshape(2, C, 5, 7)
    xn = x.clone().requires_grad_(True)
    y = OF.channel_shuffle(xn, g)
    assert torch.equal(y.float(), ref.detach())
    dy = torch.randn_like(ref).bfloat16()
    ref.backward(dy.float())
    y.backward(dy.contiguous(memory_format=torch.channels_last))
    assert torch.equal(xn.grad.float(), xr.grad)


def test_chan_remap_row_map_and_accumulate():
    """chan_remap with an outer row map (conv weight padding) and fp32 accumulation vs indexing."""
    from pytorch_cifar_amd import _native

    C = _native.lib()
    torch.manual_seed(19)
    K, Cin = 9, 13
    x = torch.randn(6 * K, Cin, device="cuda")
    cmap = [c if c < Cin else -1 for c in range(16)]
    rmap = [0, 1, -1, 2, 3, 4, 5, -1]
    out = C.chan_remap(x, torch.tensor(cmap, dtype=torch.int32, device="cuda"),
                       torch.tensor(rmap, dtype=torch.int32, device="cuda"), K)
    xv = x.view(6, K, Cin)
    ref = torch.zeros(8, K, 16, device="cuda")
    for r, s in enumerate(rmap):
        if s >= 0:
            ref[r, :, :Cin] = xv[s]
    assert torch.equal(out.view(8, K, 16), ref)
    acc = torch.ones(8 * K, 16, device="cuda")
    C.chan_remap(x, torch.tensor(cmap, dtype=torch.int32, device="cuda"),
                 torch.tensor(rmap, dtype=torch.int32, device="cuda"), K, acc)
    assert torch.allclose(acc.view(8, K, 16), ref + 1)


def test_dpn_merge_matches_torch():
    """Native DPN dual-path join vs relu(cat[x[:d] + o[:d], x[d:], o[d:]]) and its gradients."""
    from pytorch_cifar_amd.ops import functional as OF

    torch.manual_seed(8)
    d = 64
    x = torch.randn(3, 80, 6, 6, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    o = torch.randn(3, 96, 6, 6, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xr, orr = x.float().requires_grad_(True), o.float().requires_grad_(True)
    ref = torch.relu(torch.cat([xr[:, :d] + orr[:, :d], xr[:, d:], orr[:, d:]], 1))
    xn, on = x.clone().requires_grad_(True), o.clone().requires_grad_(True)
    y = OF.dpn_merge(xn, on, d)
    assert y.shape == ref.shape and rel(y, ref) < 1e-2
    dy = torch.randn_like(ref).bfloat16()
    ref.backward(dy.float())
    y.backward(dy.contiguous(memory_format=torch.channels_last))
    assert rel(xn.grad, xr.grad) < 1e-2 and rel(on.grad, orr.grad) < 1e-2


@pytest.mark.parametrize("widths", [(32, 64), (12, 24, 36), (58, 58), (3, 5, 7)])
def test_native_channel_cat_matches_torch(widths):
    """Native NHWC channel concat / split (forward + backward) vs torch.cat."""
    from pytorch_cifar_amd.ops import functional as OF

    torch.manual_seed(9)
    xs = [torch.randn(2, w, 5, 5, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
          .requires_grad_(True) for w in widths]
    refs = [x.detach().float().requires_grad_(True) for x in xs]
    y = OF.cat(xs, 1)
    ref = torch.cat(refs, 1)
    assert torch.equal(y.float(), ref)
    dy = torch.randn_like(ref).bfloat16()
    y.backward(dy.contiguous(memory_format=torch.channels_last))
    ref.backward(dy.float())
    for x, r in zip(xs, refs):
        assert torch.equal(x.grad.float(), r.grad)


@pytest.mark.parametrize("Cin,Cout,G,k,s", [(12, 44, 1, 3, 1), (96, 96, 32, 3, 2), (3, 6, 1, 5, 1)])
def test_direct_conv_fallback_matches_fp32(Cin, Cout, G, k, s, monkeypatch):
    """The scalar direct-conv kernels (PCA_GROUP_PAD=0 fallback): y, dX, dW, db vs fp32."""
    import torch.nn.functional as F
    from pytorch_cifar_amd.ops import functional as OF

    monkeypatch.setattr(OF, "_GROUP_PAD", False)
    torch.manual_seed(10)
    p = k // 2
    x = torch.randn(2, Cin, 9, 9, device="cuda").bfloat16().float().requires_grad_(True)
    w = (torch.randn(Cout, Cin // G, k, k, device="cuda") * 0.2).requires_grad_(True)
    b = torch.randn(Cout, device="cuda").requires_grad_(True)
    ref = F.conv2d(x, w, b, s, p, 1, G)
    dy = torch.randn_like(ref).bfloat16().float()
    ref.backward(dy)
    xn = x.detach().bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wn = w.detach().clone().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    bn = b.detach().clone().requires_grad_(True)
    y, _ = OF.conv2d(xn, wn, bn, s, p, G, False)
    assert rel(y, ref) < 1e-2
    y.backward(dy.to(y.dtype))
    assert rel(xn.grad, x.grad) < 2e-2 and rel(wn.grad, w.grad) < 2e-2 and rel(bn.grad, b.grad) < 2e-2


@pytest.mark.parametrize("C", [116, 58, 7])
def test_split_and_cat_shuffle2_match_torch(C):
    """Native channel split and fused shuffle(cat([a, b]), 2) vs the torch slice / cat / view
    composition, forward and backward (bitwise: pure data movement)."""
    from pytorch_cifar_amd.ops import functional as OF

    torch.manual_seed(11)
    x = torch.randn(2, 2 * C, 4, 4, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xn, xr = x.clone().requires_grad_(True), x.float().requires_grad_(True)
    a, b = OF.split_channels(xn, C)
    ar, br = xr[:, :C], xr[:, C:]
    assert torch.equal(a.float(), ar) and torch.equal(b.float(), br)
    y = OF.cat_shuffle2(b, a)
    yr = torch.cat([br, ar], 1).view(2, 2, C, 4, 4).transpose(1, 2).reshape(2, 2 * C, 4, 4)
    assert torch.equal(y.float(), yr)
    dy = torch.randn_like(yr).bfloat16()
    y.backward(dy.contiguous(memory_format=torch.channels_last))
    yr.backward(dy.float())
    assert torch.equal(xn.grad.float(), xr.grad)


@pytest.mark.parametrize("stride", [1, 2])
def test_noact_bn_fusion_matches_separate_reduce(stride, monkeypatch):
    """A BatchNorm without activation (MobileNetV2 block tail) whose backward sums are reduced by
    its consumer conv's dgrad epilogue under an all-ones mask (PCA_FUSE_BN_NOACT=1) vs the
    separate reduce + finalize passes (0): against the fp32 CPU reference, every gradient of the
    fused run is as accurate as the unfused run's."""
    from pytorch_cifar_amd.models.mobilenetv2 import Block
    from pytorch_cifar_amd.nn import Sequential
    from pytorch_cifar_amd.ops import functional as OF

    torch.manual_seed(3)
    # block tails with identity shortcuts (stride 1) and without (stride 2), each consumed by the
    # next block's expand conv (the fused consumer dgrad)
    base = Sequential(Block(24, 32, 6, stride), Block(32, 32, 6, 1), Block(32, 32, 6, 1))
    x = torch.randn(32, 24, 16, 16).bfloat16().float()
    ref = copy.deepcopy(base)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    g = torch.randn(yr.shape).bfloat16().float()
    yr.backward(g)
    want = {n: p.grad for n, p in ref.named_parameters()}
    res = {}
    for fuse in (True, False):
        m = copy.deepcopy(base).cuda().to(memory_format=torch.channels_last)
        monkeypatch.setattr(OF, "_FUSE_BN_NOACT", fuse)
        xi = x.cuda().bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
            y = m(xi)
            y.backward(g.cuda().to(y.dtype).contiguous(memory_format=torch.channels_last))
            torch.cuda.synchronize()
        reduces = sum(1 for e in prof.events() if "bn_bwd_reduce" in e.name)
        errs = {n: rel(p.grad, want[n]) for n, p in m.named_parameters()}
        res[fuse] = (rel(xi.grad, xr.grad), errs, reduces)
    assert res[True][2] < res[False][2], (res[True][2], res[False][2])   # the fusion engaged
    assert res[True][0] <= 1.5 * res[False][0] + 1e-2, (res[True][0], res[False][0])
    bad = [(n, round(e, 4), round(res[False][1][n], 4)) for n, e in res[True][1].items()
           if e > 1.5 * res[False][1][n] + 2e-2]
    assert not bad, bad


@pytest.mark.parametrize("name,kind", [("ShuffleNetV2_1", "gpad"), ("ShuffleNetG2", "gpad"),
                                       ("PNASNetA", "gpad"), ("DPN26", "gdense"),
                                       ("ResNeXt29_32x4d", "gdense")])
def test_group_padded_plan_operands_match_remap(name, kind):
    """Odd-width convs (gpad) and narrow-group super-group convs (gdense) under a WeightPrepPlan
    get their zero-padded / block-diagonal bf16 operands from the plan's batched launch
    (weight_prep pass 5 / 6, straight from the fp32 master) instead of a per-step fp32 remap +
    convert: outputs and every gradient bitwise equal to the remap path."""
    import copy

    import pytorch_cifar_amd as pca
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.ops.functional import enable_batched_weight_prep

    pca.set_deterministic(True)
    try:
        torch.manual_seed(0)
        a = models.MODEL_REGISTRY[name]().cuda().to(memory_format=torch.channels_last)
        b = copy.deepcopy(a)
        enable_batched_weight_prep(b)
        x = torch.randn(8, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        g = torch.randn(8, 10, device="cuda").to(torch.bfloat16)
        outs = []
        # three calls each, compared call by call (a call's BN statistics are shifted by the
        # previous call's batch mean, so call i of one model matches call i of the other);
        # b: the registration step, then the plan's batched refreshes
        for m in (a, a, a, b, b, b):
            m.zero_grad(set_to_none=True)
            y = m(x.clone().requires_grad_(True))
            y.backward(g)
            torch.cuda.synchronize()
            outs.append((y.detach().float(), {n: p.grad.clone() for n, p in m.named_parameters()
                                              if p.grad is not None}))
        plan = b.__dict__["_pca_wplan"]
        assert any(isinstance(e.groups, tuple) and e.groups[0] == kind for e in plan.entries)
        for e in plan.entries:     # persistent padded dW buffers are handed back all-zero
            if getattr(e, "dwbuf", None) is not None:
                assert not e.dwbuf.any(), e.groups
        for i in range(3):
            o, r = outs[3 + i], outs[i]
            assert torch.equal(o[0], r[0]), ("forward", i)
            assert o[1].keys() == r[1].keys()
            for n in o[1]:
                assert torch.equal(o[1][n], r[1][n]), (n, i)
    finally:
        pca.set_deterministic(False)


@pytest.mark.parametrize("name", ["ShuffleNetV2_1", "PNASNetA"])
def test_padded_conv_output_read_in_place(name, monkeypatch):
    """Zero-padded convs (groups == 1) hand their output to the BatchNorm as a row-strided prefix
    view, and the BN's dY comes back already padded (PCA_PAD_VIEW): forward, every gradient and
    the running statistics bitwise equal to the slice / pad passes."""
    import copy

    import pytorch_cifar_amd as pca
    from pytorch_cifar_amd import models
    from pytorch_cifar_amd.ops import functional as OF

    pca.set_deterministic(True)
    try:
        torch.manual_seed(0)
        a = models.MODEL_REGISTRY[name]().cuda().to(memory_format=torch.channels_last)
        b = copy.deepcopy(a)
        x = torch.randn(8, 3, 32, 32, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        g = torch.randn(8, 10, device="cuda").to(torch.bfloat16)
        res = []
        for m, view in ((a, False), (b, True)):
            monkeypatch.setattr(OF, "_PAD_VIEW", view)
            outs = []
            for _ in range(2):
                m.zero_grad(set_to_none=True)
                y = m(x.clone().requires_grad_(True))
                y.backward(g)
                torch.cuda.synchronize()
                outs.append((y.detach().float(), {n: p.grad.clone() for n, p in m.named_parameters()
                                                  if p.grad is not None}))
            res.append((outs, {n: t.clone() for n, t in m.named_buffers()}))
        for i in range(2):
            assert torch.equal(res[0][0][i][0], res[1][0][i][0]), ("forward", i)
            for n in res[0][0][i][1]:
                assert torch.equal(res[0][0][i][1][n], res[1][0][i][1][n]), (n, i)
        for n in res[0][1]:
            assert torch.equal(res[0][1][n], res[1][1][n]), n
    finally:
        pca.set_deterministic(False)


def test_conv_bias_grad_from_bn_backward():
    """Conv2d(bias) -> BatchNorm2d (googlenet.py / vgg.py): the BN backward delivers the conv's
    bias gradient from its per-channel sums (ops.functional.BiasRec) — exactly zero for a
    training-mode BN up to rounding, as the fp32 oracle's is — and every other gradient is
    unchanged; in eval mode the conv's own column-sum kernel runs and matches fp32."""
    from pytorch_cifar_amd.nn import BatchNorm2d, Conv2d, ReLU, Sequential

    torch.manual_seed(3)
    ref = Sequential(Conv2d(16, 32, 3, padding=1), BatchNorm2d(32), ReLU(True))
    for train in (True, False):
        ref.train(train)
        nat = copy.deepcopy(ref).cuda()
        x = torch.randn(8, 16, 16, 16)
        g = torch.randn(8, 32, 16, 16)
        ref.zero_grad()
        ref(x).backward(g)
        out = nat(x.cuda().contiguous(memory_format=torch.channels_last))
        out.backward(g.cuda().to(out.dtype).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
        wscale = ref[0].weight.grad.norm().item()
        db_n, db_r = nat[0].bias.grad.float().cpu(), ref[0].bias.grad
        if train:
            assert db_r.abs().max().item() < 1e-4 * wscale     # the oracle's is rounding noise
            assert db_n.abs().max().item() < 1e-4 * wscale
        else:
            # eval: db = sum dY over the batch, a random-sign sum, so the few ReLU-mask flips of a
            # bf16 conv output near zero move it by a few % against the fp32 oracle (as they move
            # the weight gradient below). Exact check: the fp32 sum of dY under the native mask
            bn = nat[1]
            s = (bn.weight / torch.sqrt(bn.running_var + bn.eps)).detach().float()
            m = (out.detach().float() > 0).float()
            db_o = (g.cuda().to(out.dtype).float() * m * s.view(1, -1, 1, 1)).sum((0, 2, 3)).cpu()
            assert rel(db_n, db_o) < 1e-2
            assert rel(db_n, db_r) < 6e-2
        # (bf16 through a training-mode BN backward at batch 8: a few % like the stock bf16 path)
        assert rel(nat[0].weight.grad, ref[0].weight.grad) < 6e-2
        assert rel(nat[1].weight.grad, ref[1].weight.grad) < 6e-2
