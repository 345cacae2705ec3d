"""Numerics of every hand-written gfx950 kernel against a plain PyTorch fp32 reference.

The kernels are called through the raw extension (``pytorch_cifar_amd._C``) so a failure
points at the kernel, not at the autograd wiring (that is covered by test_ops_gpu.py).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    from pytorch_cifar_amd import _native

    return _native.lib()


def rel_err(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def bf(x):
    return x.to(torch.bfloat16).float()


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2).contiguous()


CONV_CASES = [
    # N, Cin, H, Cout, k, s, p, groups
    (4, 64, 32, 64, 3, 1, 1, 1),
    (2, 64, 32, 128, 3, 2, 1, 1),
    (2, 64, 32, 128, 1, 2, 0, 1),
    (3, 8, 32, 64, 3, 1, 1, 1),
    (2, 8, 32, 32, 3, 1, 1, 1),     # stem forward kernel (stem.hip), Cout 32 / 16
    (5, 8, 32, 16, 3, 1, 1, 1),
    (3, 32, 16, 96, 3, 1, 1, 1),
    (2, 128, 8, 256, 3, 1, 1, 1),
    (5, 256, 4, 512, 3, 1, 1, 1),
    (2, 64, 16, 64, 3, 1, 1, 2),
    (2, 32, 8, 32, 3, 2, 1, 4),
    (2, 96, 8, 576, 1, 1, 0, 1),
    (2, 24, 16, 16, 1, 1, 0, 1),
    # 1x1 with reduction widths not a multiple of 64 (fast path, partial last K-step)
    (3, 144, 16, 24, 1, 1, 0, 1),
    (2, 160, 8, 320, 1, 2, 0, 1),
    (2, 48, 8, 96, 1, 1, 0, 2),
    (2, 40, 8, 200, 1, 1, 0, 1),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(C, case):
    N, Cin, H, Cout, k, s, p, G = case
    torch.manual_seed(0)
    x = bf(torch.randn(N, Cin, H, H, device="cuda"))
    w = bf(torch.randn(Cout, Cin // G, k, k, device="cuda") * (2.0 / (Cin // G * k * k)) ** 0.5)
    x.requires_grad_(True)
    w.requires_grad_(True)
    ref = F.conv2d(x, w, stride=s, padding=p, groups=G)
    dy = bf(torch.randn_like(ref))
    ref.backward(dy)

    x_n = nhwc(x.detach()).to(torch.bfloat16)
    w_p = w.detach().permute(0, 2, 3, 1).contiguous()  # [Cout, KH, KW, Cin/G] fp32
    wb, wt = C.weight_prep(w_p, G, True)
    y, stats = C.conv_fwd(x_n, wb, None, s, p, G, True)
    assert rel_err(nchw(y), ref) < 2e-2
    ssum = stats[:, 0, :].sum(0)
    ssq = stats[:, 1, :].sum(0)
    assert rel_err(ssum, ref.detach().sum((0, 2, 3))) < 2e-3 + 1e-2
    assert rel_err(ssq, (ref.detach() ** 2).sum((0, 2, 3))) < 1e-2

    dy_n = nhwc(dy).to(torch.bfloat16)
    dx = C.conv_dgrad(dy_n, wt, H, H, s, p, G)
    assert rel_err(nchw(dx), x.grad) < 2e-2
    # fused gradient hand-off: dX + addend in the epilogue (or the split-K reduce)
    add = torch.randn_like(dx)
    dx2 = C.conv_dgrad(dy_n, wt, H, H, s, p, G, add)
    assert rel_err(nchw(dx2).float(), x.grad + nchw(add).float()) < 2e-2
    dw = C.conv_wgrad(x_n, dy_n, k, k, s, p, G, None)
    assert rel_err(dw.permute(0, 3, 1, 2), w.grad) < 2e-2


N_IGEMM_CFGS = 19


@pytest.mark.parametrize("case", [(3, 64, 16, 64, 3, 1, 1, 1), (2, 128, 8, 256, 3, 2, 1, 1),
                                  (2, 32, 8, 64, 3, 1, 1, 1), (3, 64, 7, 128, 3, 1, 1, 2),
                                  (2, 64, 8, 128, 1, 2, 0, 1), (5, 128, 16, 320, 3, 1, 1, 1),
                                  (9, 256, 8, 256, 3, 1, 1, 1)])
def test_conv_every_tile_config(C, case):
    """Every compiled fwd/dgrad tile configuration (4- and 8-wave, fast scalar-tap path for
    Cin % 64 == 0 and the generic gather otherwise, stride-2 parity dgrad, odd M tails)."""
    N, Cin, H, Cout, k, s, p, G = case
    torch.manual_seed(1)
    x = bf(torch.randn(N, Cin, H, H, device="cuda"))
    w = bf(torch.randn(Cout, Cin // G, k, k, device="cuda") * (2.0 / (Cin // G * k * k)) ** 0.5)
    x.requires_grad_(True)
    ref = F.conv2d(x, w, stride=s, padding=p, groups=G)
    dy = bf(torch.randn_like(ref))
    ref.backward(dy)
    x_n = nhwc(x.detach()).to(torch.bfloat16)
    wb, wt = C.weight_prep(w.permute(0, 2, 3, 1).contiguous(), G, True)
    dy_n = nhwc(dy).to(torch.bfloat16)
    bad = []
    try:
        for cfg in list(range(N_IGEMM_CFGS)) + [20, 21, 22, 23]:   # 20-23: phased 256-row kernel
            for split in (0, 3):   # 0: no split-K; 3: K loop split 3 ways + reduce kernel
                C.set_conv_tile(0, cfg)
                C.set_conv_tile(2, split)
                y, stats = C.conv_fwd(x_n, wb, None, s, p, G, True)
                dx = C.conv_dgrad(dy_n, wt, H, H, s, p, G)
                e1, e2 = rel_err(nchw(y), ref), rel_err(nchw(dx), x.grad)
                e3 = rel_err(stats[:, 0, :].sum(0), ref.detach().sum((0, 2, 3)))
                if e1 > 2e-2 or e2 > 2e-2 or e3 > 1.2e-2:
                    bad.append((cfg, split, e1, e2, e3))
    finally:
        C.set_conv_tile(0, -1)
        C.set_conv_tile(2, -1)
    assert not bad, bad


@pytest.mark.parametrize("case", [(4, 128, 16, 128), (8, 256, 8, 256), (8, 128, 8, 256),
                                  (16, 512, 4, 512), (8, 256, 4, 128), (12, 128, 16, 256)])
def test_conv3x3_halo_kernel(C, case):
    """Halo-staged 3x3 s1 kernel (conv3x3_hx.hip, cfg 30) for layers 2-4: forward (+BN sums,
    +bias), dgrad, and dgrad with the fused residual addend + BatchNorm-backward reduce, against
    fp32 torch."""
    N, Cin, H, Cout = case
    torch.manual_seed(4)
    x = bf(torch.randn(N, Cin, H, H, device="cuda")).requires_grad_(True)
    w = bf(torch.randn(Cout, Cin, 3, 3, device="cuda") * (2.0 / (Cin * 9)) ** 0.5)
    b = torch.randn(Cout, device="cuda") * 0.1
    ref = F.conv2d(x, w, padding=1)
    dy = bf(torch.randn_like(ref))
    ref.backward(dy)
    x_n = nhwc(x.detach()).to(torch.bfloat16)
    wb, wt = C.weight_prep(w.permute(0, 2, 3, 1).contiguous(), 1, True)
    dy_n = nhwc(dy).to(torch.bfloat16)
    # BN(+ReLU) that produced x: y, 1-bit mask, mean | istd (for the fused backward reduce)
    ybn = torch.randn(N, H, H, Cin, device="cuda").to(torch.bfloat16)
    mask_b = torch.rand(N, H, H, Cin, device="cuda") > 0.4
    bits = (mask_b.view(-1, 8).to(torch.int32) << torch.arange(8, device="cuda")).sum(1).to(torch.uint8)
    mean, istd = torch.randn(Cin, device="cuda") * 0.1, torch.rand(Cin, device="cuda") + 0.5
    aux = torch.cat([mean, istd])
    add = torch.randn(N, H, H, Cin, device="cuda").to(torch.bfloat16)
    try:
        C.set_conv_tile(0, 30)
        y, stats = C.conv_fwd(x_n, wb, None, 1, 1, 1, True)
        assert rel_err(nchw(y), ref) < 2e-2
        assert rel_err(stats[:, 0, :].sum(0), ref.detach().sum((0, 2, 3))) < 1e-2
        assert rel_err(stats[:, 1, :].sum(0), (ref.detach() ** 2).sum((0, 2, 3))) < 1e-2
        yb, _ = C.conv_fwd(x_n, wb, b, 1, 1, 1, False)
        assert rel_err(nchw(yb), ref + b[None, :, None, None]) < 2e-2
        dx = C.conv_dgrad(dy_n, wt, H, H, 1, 1, 1)
        assert rel_err(nchw(dx), x.grad) < 2e-2
        dx2, part = C.conv_dgrad_bn(dy_n, wt, H, H, 1, 1, 1, add, ybn, bits, aux)
        full = nhwc(x.grad) + add.float()
        assert rel_err(dx2, full) < 2e-2
        dz = torch.where(mask_b, dx2.float(), torch.zeros_like(full))
        s1 = dz.sum((0, 1, 2))
        s2 = (dz * (ybn.float() - mean) * istd).sum((0, 1, 2))
        assert part.numel() > 0
        assert rel_err(part[:, 0, :].sum(0), s1) < 1e-2 and rel_err(part[:, 1, :].sum(0), s2) < 1e-2
    finally:
        C.set_conv_tile(0, -1)


@pytest.mark.parametrize("ver", [2, 3, 4])
@pytest.mark.parametrize("N", [4, 9])
def test_conv3x3_c64_versions(C, ver, N):
    """Layer-1 c64 kernel (conv3x3_c64.hip): v2 (16x16x32 MFMA) and v3 (32x32x16, plane LDS
    layout, DPP-paired forward sums) — forward with slab and shifted-accumulator statistics, dgrad
    with the residual addend + fused BatchNorm-backward reduce (slab and accumulator), vs fp32.
    N = 9: 36 tiles, so some persistent workgroups run an odd number of tiles (deferred epilogue
    of the last tile from either accumulator set)."""
    H, Cc = 32, 64
    torch.manual_seed(7)
    x = bf(torch.randn(N, Cc, H, H, device="cuda")).requires_grad_(True)
    w = bf(torch.randn(Cc, Cc, 3, 3, device="cuda") * (2.0 / (Cc * 9)) ** 0.5)
    ref = F.conv2d(x, w, padding=1)
    dy = bf(torch.randn_like(ref))
    ref.backward(dy)
    x_n = nhwc(x.detach()).to(torch.bfloat16)
    wb, wt = C.weight_prep(w.permute(0, 2, 3, 1).contiguous(), 1, True)
    dy_n = nhwc(dy).to(torch.bfloat16)
    ybn = torch.randn(N, H, H, Cc, device="cuda").to(torch.bfloat16)
    mask_b = torch.rand(N, H, H, Cc, device="cuda") > 0.4
    bits = (mask_b.view(-1, 8).to(torch.int32) << torch.arange(8, device="cuda")).sum(1).to(torch.uint8)
    mean, istd = torch.randn(Cc, device="cuda") * 0.1, torch.rand(Cc, device="cuda") + 0.5
    aux = torch.cat([mean, istd])
    add = torch.randn(N, H, H, Cc, device="cuda").to(torch.bfloat16)
    r = ref.detach()
    prev = C.c64_version(ver)
    try:
        y, stats = C.conv_fwd(x_n, wb, None, 1, 1, 1, True)
        assert rel_err(nchw(y), r) < 2e-2
        assert rel_err(stats[:, 0, :].sum(0), r.sum((0, 2, 3))) < 1e-2
        assert rel_err(stats[:, 1, :].sum(0), (r ** 2).sum((0, 2, 3))) < 1e-2
        # shifted sums into a 4-row accumulator (+ its K row)
        K = torch.randn(Cc, device="cuda")
        R = 4
        acc = torch.zeros(R * 2 * Cc + Cc, device="cuda")
        y2, _ = C.conv_fwd(x_n, wb, None, 1, 1, 1, True, acc, R, K)
        assert torch.equal(y2, y)
        a = acc[:R * 2 * Cc].view(R, 2, Cc).sum(0)
        yf = y.float().reshape(-1, Cc)
        d = r.permute(0, 2, 3, 1).reshape(-1, Cc) - K
        assert rel_err(a[0], d.sum(0)) < 1e-2
        assert rel_err(a[1], (d ** 2).sum(0)) < 1e-2
        assert torch.equal(acc[R * 2 * Cc:], K)
        dx = C.conv_dgrad(dy_n, wt, H, H, 1, 1, 1)
        assert rel_err(nchw(dx), x.grad) < 2e-2
        full = nhwc(x.grad) + add.float()
        dz_ref = None
        for use_acc in (False, True):
            if use_acc:
                bacc = torch.zeros(R * 2 * Cc, device="cuda")
                dx2, part = C.conv_dgrad_bn(dy_n, wt, H, H, 1, 1, 1, add, ybn, bits, aux, bacc, R)
                part = bacc.view(R, 2, Cc)
            else:
                dx2, part = C.conv_dgrad_bn(dy_n, wt, H, H, 1, 1, 1, add, ybn, bits, aux)
            assert rel_err(dx2, full) < 2e-2
            dz = torch.where(mask_b, dx2.float(), torch.zeros_like(full))
            s1 = dz.sum((0, 1, 2))
            s2 = (dz * (ybn.float() - mean) * istd).sum((0, 1, 2))
            assert part.numel() > 0
            assert rel_err(part[:, 0, :].sum(0), s1) < 1e-2 and rel_err(part[:, 1, :].sum(0), s2) < 1e-2
        del yf, dz_ref
    finally:
        C.c64_version(prev)


@pytest.mark.parametrize("case", [(4, 64, 32, 128), (8, 128, 16, 256), (16, 256, 8, 512),
                                  (8, 32, 16, 64), (4, 96, 32, 64)])
def test_conv3x3_s2_dgrad_halo_kernel(C, case):
    """Stride-2 dgrad through the halo kernel (cfg 30, mode 2): a 2x2 convolution over dY whose
    4 x Cin output channels are the four parity classes of dX, written depth-to-space; plain,
    and with the fused residual addend + BatchNorm-backward reduce, against fp32 torch."""
    N, Cin, H, Cout = case
    torch.manual_seed(5)
    x = bf(torch.randn(N, Cin, H, H, device="cuda")).requires_grad_(True)
    w = bf(torch.randn(Cout, Cin, 3, 3, device="cuda") * (2.0 / (Cin * 9)) ** 0.5)
    ref = F.conv2d(x, w, stride=2, padding=1)
    dy = bf(torch.randn_like(ref))
    ref.backward(dy)
    wb, wt = C.weight_prep(w.permute(0, 2, 3, 1).contiguous(), 1, True)
    dy_n = nhwc(dy).to(torch.bfloat16)
    ybn = torch.randn(N, H, H, Cin, device="cuda").to(torch.bfloat16)
    mask_b = torch.rand(N, H, H, Cin, device="cuda") > 0.4
    bits = (mask_b.view(-1, 8).to(torch.int32) << torch.arange(8, device="cuda")).sum(1).to(torch.uint8)
    mean, istd = torch.randn(Cin, device="cuda") * 0.1, torch.rand(Cin, device="cuda") + 0.5
    aux = torch.cat([mean, istd])
    add = torch.randn(N, H, H, Cin, device="cuda").to(torch.bfloat16)
    try:
        C.set_conv_tile(0, 30)
        dx = C.conv_dgrad(dy_n, wt, H, H, 2, 1, 1)
        assert rel_err(nchw(dx), x.grad) < 2e-2
        dx2, part = C.conv_dgrad_bn(dy_n, wt, H, H, 2, 1, 1, add, ybn, bits, aux)
        full = nhwc(x.grad) + add.float()
        assert rel_err(dx2, full) < 2e-2
        dz = torch.where(mask_b, dx2.float(), torch.zeros_like(full))
        s1 = dz.sum((0, 1, 2))
        s2 = (dz * (ybn.float() - mean) * istd).sum((0, 1, 2))
        assert part.numel() > 0
        assert rel_err(part[:, 0, :].sum(0), s1) < 1e-2 and rel_err(part[:, 1, :].sum(0), s2) < 1e-2
    finally:
        C.set_conv_tile(0, -1)


@pytest.mark.parametrize("case", [(2, 64, 16, 64, 3, 1, 1, 1), (3, 128, 8, 256, 3, 2, 1, 1),
                                  (2, 64, 16, 128, 1, 2, 0, 1), (2, 128, 8, 128, 3, 1, 1, 2)])
def test_wgrad_autotune_candidates(C, case):
    """Every (config, forced split-K) candidate the wgrad autotuner may pick is numerically right."""
    N, Cin, H, Cout, k, s, p, G = case
    torch.manual_seed(2)
    x = bf(torch.randn(N, Cin, H, H, device="cuda"))
    w = bf(torch.randn(Cout, Cin // G, k, k, device="cuda") * 0.05).requires_grad_(True)
    ref = F.conv2d(x, w, stride=s, padding=p, groups=G)
    dy = bf(torch.randn_like(ref))
    ref.backward(dy)
    x_n = nhwc(x).to(torch.bfloat16)
    dy_n = nhwc(dy).to(torch.bfloat16)
    cands = C.wgrad_candidates(N, H, H, Cin, Cout, k, k, s, p, G)
    assert len(cands) > 6
    bad = []
    try:
        for cfg, split in cands:
            C.conv_trial(1, cfg, split)
            dw = C.conv_wgrad(x_n, dy_n, k, k, s, p, G, None)
            e = rel_err(dw.permute(0, 3, 1, 2), w.grad)
            if e > 2e-2:
                bad.append((cfg, split, e))
    finally:
        C.conv_trial(1, -1, -1)
    assert not bad, bad


WGRAD_CFGS = list(range(8)) + list(range(16, 22)) + list(range(32, 47))   # 39-41: one kernel row (3 taps) per halo tile; 42-46: 4-6 LDS stages


@pytest.mark.parametrize("case", [(3, 64, 16, 64, 3, 1, 1, 1), (2, 128, 8, 256, 3, 2, 1, 1),
                                  (2, 64, 32, 128, 1, 2, 0, 1), (3, 128, 7, 64, 3, 1, 1, 2),
                                  (4, 64, 4, 192, 3, 1, 1, 1), (3, 64, 32, 64, 3, 1, 1, 1),
                                  (5, 128, 8, 128, 3, 1, 1, 2), (64, 64, 32, 64, 3, 1, 1, 1)])
def test_wgrad_every_config(C, case):
    """Every wgrad configuration: split-K atomics, wide slab kernels (deterministic) and their
    column / channel tails, accumulating into an existing gradient."""
    N, Cin, H, Cout, k, s, p, G = case
    torch.manual_seed(2)
    x = bf(torch.randn(N, Cin, H, H, device="cuda"))
    w = bf(torch.randn(Cout, Cin // G, k, k, device="cuda") * 0.1).requires_grad_(True)
    ref = F.conv2d(x, w, stride=s, padding=p, groups=G)
    dy = bf(torch.randn_like(ref))
    ref.backward(dy)
    x_n = nhwc(x).to(torch.bfloat16)
    dy_n = nhwc(dy).to(torch.bfloat16)
    prev = torch.randn(Cout, k, k, Cin // G, device="cuda")
    want = w.grad.permute(0, 2, 3, 1) + prev
    bad = []
    try:
        for cfg in WGRAD_CFGS:
            C.set_conv_tile(1, cfg)
            dw = C.conv_wgrad(x_n, dy_n, k, k, s, p, G, prev.clone())
            e = rel_err(dw, want)
            if e > 2e-2:
                bad.append((cfg, e))
        C.set_conv_tile(1, 16)
        a = C.conv_wgrad(x_n, dy_n, k, k, s, p, G, None)
        b = C.conv_wgrad(x_n, dy_n, k, k, s, p, G, None)
    finally:
        C.set_conv_tile(1, -1)
    assert not bad, bad


@pytest.mark.parametrize("C_,act,res", [(64, 1, False), (64, 1, True), (24, 0, False), (116, 1, True), (96, 2, False),
                                        (58, 1, False), (44, 2, False), (7, 1, True), (58, 0, True)])
def test_bn_fwd_bwd(C, C_, act, res):
    torch.manual_seed(1)
    N, H = 4, 8
    y = bf(torch.randn(N, C_, H, H, device="cuda") * 2 + 0.5).requires_grad_(True)
    r = bf(torch.randn(N, C_, H, H, device="cuda")).requires_grad_(True) if res else None
    gamma = torch.rand(C_, device="cuda").add_(0.5).requires_grad_(True)
    beta = torch.randn(C_, device="cuda").requires_grad_(True)
    rm_ref = torch.zeros(C_, device="cuda")
    rv_ref = torch.ones(C_, device="cuda")
    z = F.batch_norm(y, rm_ref, rv_ref, gamma, beta, training=True, momentum=0.1, eps=1e-5)
    if res:
        z = z + r
    out_ref = F.relu(z) if act == 1 else (F.silu(z) if act == 2 else z)
    dout = bf(torch.randn_like(out_ref))
    out_ref.backward(dout)

    yn = nhwc(y.detach()).to(torch.bfloat16)
    rn = nhwc(r.detach()).to(torch.bfloat16) if res else None
    rm = torch.zeros(C_, device="cuda")
    rv = torch.ones(C_, device="cuda")
    nbt = torch.zeros((), dtype=torch.long, device="cuda")
    partial = C.bn_stats(yn)
    aux = C.bn_finalize(partial, float(N * H * H), gamma.detach(), beta.detach(), rm, rv, nbt, 0.1, 1e-5, True, True)
    out, mask = C.bn_apply(yn, aux, rn, None, None, act, act == 1)
    assert rel_err(nchw(out), out_ref) < 2e-2
    if act == 1 and C_ % 8 == 0:   # ReLU sign bits, one byte per 8 channels
        bits = ((mask.view(-1, 1).int() >> torch.arange(8, device="cuda")) & 1).view(-1)
        assert torch.equal(bits.bool(), (out.reshape(-1) > 0))
    assert rel_err(rm, rm_ref) < 1e-4 and rel_err(rv, rv_ref) < 1e-4
    assert nbt.item() == 1
    dn = nhwc(dout).to(torch.bfloat16)
    use_mask = mask is not None and mask.numel() > 0
    dy, dres, _, dg, db, _, _ = C.bn_backward(dn, None if use_mask else out, mask if use_mask else None, yn, aux,
                                              gamma.detach(), None, None, None, act, True, res, None, None, None, None)
    assert rel_err(nchw(dy), y.grad) < 3e-2
    assert rel_err(dg, gamma.grad) < 1e-2
    assert rel_err(db, beta.grad) < 1e-2
    if res:
        assert rel_err(nchw(dres), r.grad) < 2e-2


def test_bn_dual_shortcut(C):
    torch.manual_seed(2)
    N, Ch, H = 4, 64, 8
    y1 = bf(torch.randn(N, Ch, H, H, device="cuda")).requires_grad_(True)
    y2 = bf(torch.randn(N, Ch, H, H, device="cuda") * 3).requires_grad_(True)
    g1 = torch.rand(Ch, device="cuda").add_(0.5).requires_grad_(True)
    b1 = torch.randn(Ch, device="cuda").requires_grad_(True)
    g2 = torch.rand(Ch, device="cuda").add_(0.5).requires_grad_(True)
    b2 = torch.randn(Ch, device="cuda").requires_grad_(True)
    z = F.batch_norm(y1, None, None, g1, b1, training=True) + F.batch_norm(y2, None, None, g2, b2, training=True)
    out_ref = F.relu(z)
    dout = bf(torch.randn_like(out_ref))
    out_ref.backward(dout)
    cnt = float(N * H * H)
    y1n, y2n = nhwc(y1.detach()).bfloat16(), nhwc(y2.detach()).bfloat16()
    z_ = torch.zeros(Ch, device="cuda")
    o_ = torch.ones(Ch, device="cuda")
    a1 = C.bn_finalize(C.bn_stats(y1n), cnt, g1.detach(), b1.detach(), z_.clone(), o_.clone(), None, 0.1, 1e-5, True, False)
    a2 = C.bn_finalize(C.bn_stats(y2n), cnt, g2.detach(), b2.detach(), z_.clone(), o_.clone(), None, 0.1, 1e-5, True, False)
    out, _ = C.bn_apply(y1n, a1, None, y2n, a2, 1, False)
    assert rel_err(nchw(out), out_ref) < 2e-2
    dy1, _, dy2, dg1, db1, dg2, db2 = C.bn_backward(nhwc(dout).bfloat16(), out, None, y1n, a1, g1.detach(), y2n, a2, g2.detach(), 1, True, False, None, None, None, None)
    assert rel_err(nchw(dy1), y1.grad) < 3e-2
    assert rel_err(nchw(dy2), y2.grad) < 3e-2
    assert rel_err(dg1, g1.grad) < 1e-2 and rel_err(dg2, g2.grad) < 1e-2
    assert rel_err(db1, b1.grad) < 1e-2 and rel_err(db2, b2.grad) < 1e-2


def test_cross_entropy(C):
    torch.manual_seed(3)
    logits = torch.randn(300, 10, device="cuda").requires_grad_(True)
    tgt = torch.randint(0, 10, (300,), device="cuda")
    ref = F.cross_entropy(logits, tgt)
    ref.backward()
    metrics = torch.zeros(3, dtype=torch.float64, device="cuda")
    loss, dl = C.ce_fused(logits.detach(), tgt, metrics, True)
    assert abs(loss.item() - ref.item()) < 1e-4
    assert rel_err(dl, logits.grad) < 1e-4
    correct = (logits.argmax(1) == tgt).sum().item()
    assert metrics[1].item() == correct and metrics[2].item() == 300


@pytest.mark.parametrize("K", [10, 40])
def test_cross_entropy_bad_label_poisons(C, K):
    """A label outside [0, K) must not train silently (F.cross_entropy raises): the fused kernel
    NaN-poisons the loss and that sample's gradient row (register path K<=16 and row path)."""
    logits = torch.randn(64, K, device="cuda")
    tgt = torch.randint(0, K, (64,), device="cuda")
    tgt[5] = K
    tgt[9] = -1
    loss, dl = C.ce_fused(logits, tgt, None, True)
    assert torch.isnan(loss).all()
    assert torch.isnan(dl[5]).all() and torch.isnan(dl[9]).all()
    assert torch.isfinite(dl[0]).all()


@pytest.mark.parametrize("Cc", [16, 12])
def test_pools_and_gap(C, Cc):
    """Max/avg pools and global average pool; C % 8 == 0 takes the vectorized max-pool kernels."""
    torch.manual_seed(4)
    x = bf(torch.randn(2, Cc, 8, 8, device="cuda")).requires_grad_(True)
    xn = nhwc(x.detach()).bfloat16()
    for k, s, p in [(2, 2, 0), (3, 1, 1), (3, 2, 1)]:
        ref = F.max_pool2d(x, k, s, p)
        dy = bf(torch.randn_like(ref))
        (g,) = torch.autograd.grad(ref, x, dy)
        y, arg = C.maxpool_fwd(xn, k, s, p)
        assert rel_err(nchw(y), ref) < 1e-2
        dx = C.maxpool_bwd(nhwc(dy).bfloat16(), arg, 8, 8, k, s, p)
        assert rel_err(nchw(dx), g) < 1e-2
    for k, s, p in [(2, 2, 0), (4, 4, 0), (3, 2, 1)]:
        ref = F.avg_pool2d(x, k, s, p)
        dy = bf(torch.randn_like(ref))
        (g,) = torch.autograd.grad(ref, x, dy)
        y = C.avgpool_fwd(xn, k, s, p)
        assert rel_err(nchw(y), ref) < 1e-2
        dx = C.avgpool_bwd(nhwc(dy).bfloat16(), 8, 8, k, s, p)
        assert rel_err(nchw(dx), g) < 1e-2
    pooled = C.gap_fwd(xn)
    assert rel_err(pooled, x.detach().mean((2, 3))) < 1e-2


@pytest.mark.parametrize("Cin,mult,k,s,H", [(32, 1, 3, 1, 16), (144, 1, 3, 2, 16), (240, 1, 5, 1, 16),
                                            (44, 2, 7, 2, 16), (58, 1, 3, 2, 16), (96, 1, 3, 1, 16),
                                            (1152, 1, 3, 1, 4), (192, 1, 3, 2, 8), (72, 1, 3, 2, 7),
                                            (24, 1, 3, 1, 9), (144, 1, 5, 2, 16), (36, 1, 5, 1, 8),
                                            (1152, 1, 5, 1, 2), (672, 1, 5, 2, 4), (2304, 1, 3, 1, 4),
                                            (20, 1, 5, 1, 6), (44, 1, 7, 1, 8), (88, 1, 7, 2, 8),
                                            (176, 1, 7, 1, 4), (30, 1, 7, 2, 9), (58, 1, 3, 1, 8),
                                            (116, 1, 3, 2, 8), (58, 1, 5, 1, 6), (26, 1, 3, 1, 5),
                                            (96, 1, 3, 1, 32), (144, 1, 3, 1, 32), (200, 1, 3, 1, 12),
                                            (144, 1, 3, 2, 32), (960, 1, 3, 1, 4)])
def test_depthwise(C, Cin, mult, k, s, H):
    """Multiplier 1, k3/k5/k7, even C takes the rolling-window fast paths (8/4/2 channels per thread)
    (dwk_*, incl. > 256 channel groups split over grid.y in wgrad), the rest the generic
    kernels; both against torch's fp32 grouped conv."""
    torch.manual_seed(5)
    N = 2
    p = (k - 1) // 2
    Co = Cin * mult
    x = bf(torch.randn(N, Cin, H, H, device="cuda")).requires_grad_(True)
    w = (torch.randn(Co, 1, k, k, device="cuda") * 0.3).requires_grad_(True)
    ref = F.conv2d(x, w, stride=s, padding=p, groups=Cin)
    dy = bf(torch.randn_like(ref))
    ref.backward(dy)
    wT = w.detach().reshape(Co, k * k).t().contiguous()
    xn = nhwc(x.detach()).bfloat16()
    y = C.dw_fwd(xn, wT, k, k, s, p)
    assert rel_err(nchw(y), ref) < 2e-2
    dx = C.dw_dgrad(nhwc(dy).bfloat16(), wT, H, H, Cin, k, k, s, p)
    assert rel_err(nchw(dx), x.grad) < 2e-2
    dw = C.dw_wgrad(xn, nhwc(dy).bfloat16(), k, k, s, p)
    assert rel_err(dw.reshape(Co, 1, k, k), w.grad) < 2e-2


@pytest.mark.parametrize("Cin,k,s,H,N", [(96, 3, 1, 16, 4), (144, 3, 2, 16, 3), (240, 3, 1, 8, 4),
                                          (672, 3, 2, 8, 2), (1152, 3, 1, 4, 8), (40, 3, 2, 9, 2)])
def test_depthwise_fused_bn_epilogues(C, Cin, k, s, H, N):
    """Depthwise kernels with the BatchNorm sums fused (sharded accumulator rows): the forward's
    statistics of its output, and the dgrad's backward reduce of the BN(+ReLU / swish) that
    produced its input, against fp32 sums of the same kernel's outputs; plain outputs unchanged."""
    from pytorch_cifar_amd.ops.functional import acc_shards

    torch.manual_seed(8)
    p = (k - 1) // 2
    x = bf(torch.randn(N, Cin, H, H, device="cuda"))
    w = torch.randn(Cin, 1, k, k, device="cuda") * 0.3
    wT = w.reshape(Cin, k * k).t().contiguous()
    xn = nhwc(x).bfloat16()
    R = acc_shards(Cin)
    acc = torch.zeros(R * 2 * Cin, device="cuda")
    y, ok = C.dw_fwd_stats(xn, wT, k, k, s, p, acc, R)
    assert int(ok) == 1
    # (same arithmetic as the plain kernel; register allocation may contract it differently)
    assert rel_err(y, C.dw_fwd(xn, wT, k, k, s, p)) < 1e-2
    sums = acc.view(R, 2, Cin).sum(0)
    # (the epilogue sums the fp32 results before rounding: compare with the fp32 conv)
    yf = nhwc(F.conv2d(x.float(), w, stride=s, padding=p, groups=Cin)).reshape(-1, Cin)
    assert rel_err(sums[0], yf.sum(0)) < 1e-4 and rel_err(sums[1], (yf * yf).sum(0)) < 1e-4

    dy = torch.randn_like(y.float()).bfloat16()
    dx_ref = C.dw_dgrad(dy, wT, H, H, Cin, k, k, s, p)
    ybn = torch.randn(N, H, H, Cin, device="cuda").bfloat16()
    mean, istd = torch.randn(Cin, device="cuda") * 0.1, torch.rand(Cin, device="cuda") + 0.5
    scale, shift = torch.randn(Cin, device="cuda"), torch.randn(Cin, device="cuda") * 0.2
    aux = torch.cat([mean, istd, scale, shift])
    mask_b = torch.rand(N, H, H, Cin, device="cuda") > 0.4
    bits = (mask_b.reshape(-1, 8).to(torch.int32) << torch.arange(8, device="cuda")).sum(1).to(torch.uint8)
    xhat = (ybn.float() - mean) * istd
    for act in (1, 2):
        acc.zero_()
        dx, ok = C.dw_dgrad_bn(dy, wT, H, H, Cin, k, k, s, p, ybn, bits if act == 1 else None, aux,
                               act, acc, R)
        assert int(ok) == 1
        assert rel_err(dx, dx_ref) < 1e-2
        if act == 1:
            dz = torch.where(mask_b, dx.float(), torch.zeros_like(xhat))
        else:
            z = ybn.float() * scale + shift
            sg = torch.sigmoid(z)
            dz = dx.float() * (sg + z * sg * (1 - sg))
        sums = acc.view(R, 2, Cin).sum(0)
        assert rel_err(sums[0], dz.sum((0, 1, 2))) < 1e-3, act
        assert rel_err(sums[1], (dz * xhat).sum((0, 1, 2))) < 1e-3, act


@pytest.mark.parametrize("Cc,H", [(48, 4), (1152, 2), (96, 32), (20, 4)])
def test_se_scale(C, Cc, H):
    """Squeeze-excite scale fwd/bwd and the global average pool (fwd/bwd) it uses: vectorized
    8-channel kernels for C % 8 == 0, scalar ones otherwise."""
    torch.manual_seed(6)
    x = bf(torch.randn(3, Cc, H, H, device="cuda")).requires_grad_(True)
    s = torch.randn(3, Cc, device="cuda").requires_grad_(True)
    xn0 = nhwc(x.detach()).bfloat16()
    pooled = C.gap_fwd(xn0)
    assert rel_err(pooled, x.detach().mean((2, 3))) < 1e-2
    gy = torch.randn(3, Cc, device="cuda")
    gx = C.gap_bwd(gy, H, H)
    assert rel_err(nchw(gx).float(), (gy / (H * H))[:, :, None, None].expand(3, Cc, H, H)) < 1e-2
    ref = x * torch.sigmoid(s)[:, :, None, None]
    dy = bf(torch.randn_like(ref))
    ref.backward(dy)
    xn = nhwc(x.detach()).bfloat16()
    out = C.se_scale_fwd(xn, s.detach())
    assert rel_err(nchw(out), ref) < 1e-2
    dx, ds = C.se_scale_bwd(nhwc(dy).bfloat16(), xn, s.detach())
    assert rel_err(nchw(dx), x.grad) < 1e-2
    assert rel_err(ds, s.grad) < 1e-2


def test_layout_and_augment(C):
    torch.manual_seed(7)
    x = torch.randn(2, 3, 32, 32, device="cuda")
    y = C.nchw_to_nhwc(x, 8)
    assert y.shape == (2, 32, 32, 8)
    assert rel_err(y[..., :3].float(), nhwc(x)) < 1e-2 and y[..., 3:].abs().max().item() == 0
    back = C.nhwc_to_nchw(y, 3)
    assert rel_err(back, x) < 1e-2
    data = torch.randint(0, 256, (5, 32, 32, 3), dtype=torch.uint8, device="cuda")
    idx = torch.tensor([4, 0, 2], device="cuda")
    # word k: dy = k % 9, dx = (k // 9) % 9, flip = k // 81; (4, 4) is the identity crop,
    # sample 1 flips, sample 2 is dy = dx = 0
    rnd = torch.tensor([4 + 4 * 9, 4 + 4 * 9 + 81, 0], dtype=torch.int32, device="cuda")
    mean, std = [0.4914, 0.4822, 0.4465], [0.2023, 0.1994, 0.2010]
    out = C.augment(data, idx, rnd, 4, mean, std)
    m = torch.tensor(mean, device="cuda")
    sd = torch.tensor(std, device="cuda")
    ref0 = (data[4].float() / 255 - m) / sd
    assert rel_err(out[0, ..., :3], ref0) < 1e-2
    ref1 = (data[0].float().flip(1) / 255 - m) / sd
    assert rel_err(out[1, ..., :3], ref1) < 1e-2
    # dy=dx=0 shifts the image down/right by 4 with zero (-mean/std) padding
    ref2 = torch.nn.functional.pad(data[2].float().permute(2, 0, 1), (4, 4, 4, 4))[:, :32, :32].permute(1, 2, 0)
    ref2 = (ref2 / 255 - m) / sd
    assert rel_err(out[2, ..., :3], ref2) < 1e-2


def test_augment_packed_matches_unpacked(C):
    """Packed batch entries (sample | word << 32) give the images of the (idx, rnd) form and the
    gathered labels, in one launch."""
    torch.manual_seed(11)
    data = torch.randint(0, 256, (9, 32, 32, 3), dtype=torch.uint8, device="cuda")
    labels = torch.randint(0, 10, (9,), device="cuda")
    idx = torch.tensor([8, 0, 3, 3, 5], device="cuda")
    rnd = torch.randint(0, 162, (5,), dtype=torch.int32, device="cuda")
    mean, std = [0.4914, 0.4822, 0.4465], [0.2023, 0.1994, 0.2010]
    ref = C.augment(data, idx, rnd, 4, mean, std)
    packed = idx | (rnd.long() << 32)
    out, tg = C.augment_packed(data, labels, packed, 4, mean, std)
    assert torch.equal(out, ref)
    assert torch.equal(tg, labels[idx])


@pytest.mark.parametrize("N,Co", [(2, 64), (5, 32), (3, 16), (130, 64)])
def test_stem_wgrad_matches_fp32(C, N, Co):
    """Stem 3x3 wgrad (3 channels padded to 8, stride 1, pad 1) vs torch's fp32 weight gradient
    of the same bf16 operands; the result is ADDED to the existing gradient."""
    torch.manual_seed(N * 100 + Co)
    x = torch.zeros(N, 32, 32, 8, device="cuda", dtype=torch.bfloat16)
    x[..., :3] = torch.randn(N, 32, 32, 3, device="cuda").to(torch.bfloat16)
    dy = torch.randn(N, 32, 32, Co, device="cuda").to(torch.bfloat16)
    base = torch.randn(Co, 3, 3, 3, device="cuda")
    out = base.clone()
    assert C.stem_wgrad(x, dy, 1, 1, out)
    ref = torch.nn.grad.conv2d_weight(nchw(x[..., :3].float()), (Co, 3, 3, 3), nchw(dy.float()),
                                      stride=1, padding=1)
    assert rel_err(out - base, nhwc(ref)) < 2e-3
    # not the stem's shape -> declined (caller falls back)
    assert not C.stem_wgrad(x, dy, 2, 1, out)
    assert not C.stem_wgrad(x[:, :16].contiguous(), dy[:, :16].contiguous(), 1, 1,
                            torch.zeros(Co, 3, 3, 5, device="cuda"))


def test_sgd_multi_tensor(C):
    from pytorch_cifar_amd.engine.optim import SGD

    torch.manual_seed(8)
    ps = [torch.randn(n, device="cuda", requires_grad=True) for n in (10, 70000, 3)]
    ref = [p.detach().clone().requires_grad_(True) for p in ps]
    opt = SGD(ps, lr=0.1, momentum=0.9, weight_decay=5e-4)
    ropt = torch.optim.SGD(ref, lr=0.1, momentum=0.9, weight_decay=5e-4)
    for _ in range(3):
        for p, r in zip(ps, ref):
            g = torch.randn_like(p)
            p.grad = g.clone()
            r.grad = g.clone()
        opt.step()
        ropt.step()
    for p, r in zip(ps, ref):
        assert rel_err(p.detach(), r.detach()) < 1e-5


@pytest.mark.parametrize("case", [(8, 64, 32, 64, 3, 1, 1, 1), (4, 128, 16, 256, 3, 2, 1, 1),
                                  (16, 256, 8, 256, 3, 1, 1, 1), (2, 24, 16, 16, 1, 1, 0, 1)])
def test_wgrad_deterministic_mode_bitwise(C, case):
    """set_deterministic: every wgrad path (halo, wide, split-K) reduces through ordered slab
    rows -> two runs are bitwise identical (atomics make the default mode order-dependent)."""
    N, Cin, H, Cout, k, s, p, G = case
    torch.manual_seed(3)
    x = nhwc(torch.randn(N, Cin, H, H, device="cuda")).to(torch.bfloat16)
    Ho = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, Ho, Ho, Cout, device="cuda").to(torch.bfloat16)
    C.set_deterministic(True)
    try:
        for cfg in [-1, 3, 16, 32]:
            C.set_conv_tile(1, cfg)
            a = C.conv_wgrad(x, dy, k, k, s, p, G, None)
            b = C.conv_wgrad(x, dy, k, k, s, p, G, None)
            assert torch.equal(a, b), cfg
    finally:
        C.set_deterministic(False)
        C.set_conv_tile(1, -1)


def test_debug_sync_proxy_runs_ops():
    from pytorch_cifar_amd import _native

    _native.set_debug_sync(True)
    try:
        C = _native.lib()
        x = torch.randn(2, 8, 8, 16, device="cuda").to(torch.bfloat16)
        y = C.gap_fwd(x)
        assert y.shape[-1] == 16 and C.last_error() == ""
    finally:
        _native.set_debug_sync(False)


@pytest.mark.parametrize("N,H,C,K", [(128, 4, 512, 10), (7, 2, 1280, 10), (33, 8, 96, 16),
                                     (16, 1, 2048, 10), (5, 4, 4096, 3)])
def test_fused_head_matches_fp32(N, H, C, K, C_=None):
    """Fused global-average-pool + Linear (forward and backward, gradients accumulated into the
    given buffers) against the fp32 torch composition."""
    from pytorch_cifar_amd import _native

    C_ = _native.lib()
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    w = torch.randn(K, C, device="cuda") * 0.05
    b = torch.randn(K, device="cuda")
    logits, pooled, _ = C_.head_fwd(x, w, b)
    xr = x.float().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ref = torch.nn.functional.linear(xr.mean((1, 2)), wr, br)
    assert rel_err(logits, ref) < 1e-4
    assert rel_err(pooled, xr.detach().mean((1, 2))) < 1e-5
    dl = torch.randn(N, K, device="cuda")
    ref.backward(dl)
    dw0 = torch.randn(K, C, device="cuda")
    db0 = torch.randn(K, device="cuda")
    dwa, dba = dw0.clone(), db0.clone()
    dx, dw, db = C_.head_bwd(dl, w, pooled, H, H, dwa, dba, True)
    assert dw.data_ptr() == dwa.data_ptr() and db.data_ptr() == dba.data_ptr()
    assert rel_err(dx, xr.grad) < 1e-2
    assert rel_err(dw - dw0, wr.grad) < 1e-4
    assert rel_err(db - db0, br.grad) < 1e-5


def test_fused_head_dropout(C=None):
    """Pool + Philox dropout (p = 0.2, efficientnet.py:147-149) + Linear: keep rate, 1/(1-p)
    scaling, logits/gradients consistent with the returned keep mask, fresh masks per launch
    (the kernel advances its own step counter, also under hipGraph replay)."""
    from pytorch_cifar_amd import _native

    C_ = _native.lib()
    torch.manual_seed(1)
    N, H, Cc, K, p = 256, 2, 1280, 10, 0.2
    x = torch.randn(N, H, H, Cc, device="cuda").to(torch.bfloat16)
    w = torch.randn(K, Cc, device="cuda") * 0.05
    b = torch.randn(K, device="cuda")
    rng = torch.tensor([1234, 0, 0], dtype=torch.int64, device="cuda")
    logits, pooled, mask = C_.head_fwd(x, w, b, p, rng)
    keep = mask.bool()
    rate = keep.float().mean().item()
    assert abs(rate - (1 - p)) < 0.01, rate
    mean = x.float().mean((1, 2))
    assert rel_err(pooled, torch.where(keep, mean / (1 - p), torch.zeros_like(mean))) < 1e-5
    assert rel_err(logits, pooled @ w.t() + b) < 1e-4
    assert rng.tolist() == [1234, 1, 0]
    dl = torch.randn(N, K, device="cuda")
    dx, dw, db = C_.head_bwd(dl, w, pooled, H, H, None, None, True, p, mask)
    dfeat = torch.where(keep, (dl @ w) / (1 - p), torch.zeros(N, Cc, device="cuda")) / (H * H)
    assert rel_err(dx.float(), dfeat[:, None, None, :].expand(N, H, H, Cc)) < 1e-2
    assert rel_err(dw, dl.t() @ pooled) < 1e-4 and rel_err(db, dl.sum(0)) < 1e-5
    # per-step masks differ; graph replays advance the counter too
    _, _, mask2 = C_.head_fwd(x, w, b, p, rng)
    assert not torch.equal(mask, mask2) and rng.tolist() == [1234, 2, 0]
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            out = C_.head_fwd(x, w, b, p, rng)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    m3 = out[2].clone()
    g.replay()
    torch.cuda.synchronize()
    assert not torch.equal(m3, out[2]) and rng.tolist()[1] >= 4 and rng.tolist()[2] == 0


@pytest.mark.parametrize("unit", [1, 4 * 4 * 96])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_dropout_and_drop_connect(C, unit, dt):
    """Generic Philox dropout (unit 1) and per-sample drop-connect (unit = C*H*W)."""
    N, p = 512, 0.3
    x = torch.randn(N, 4, 4, 96, device="cuda").to(dt)
    rng = torch.tensor([77, 5, 0], dtype=torch.int64, device="cuda")
    y, mask = C.dropout_fwd(x, p, unit, rng)
    assert mask.numel() == x.numel() // unit and rng.tolist() == [77, 6, 0]
    keep = mask.bool().repeat_interleave(unit).view_as(x)
    assert abs(mask.float().mean().item() - (1 - p)) < (0.01 if unit == 1 else 0.06)
    ref = torch.where(keep, x.float() / (1 - p), torch.zeros_like(x, dtype=torch.float32))
    assert rel_err(y, ref) < 1e-2
    dy = torch.randn_like(x)
    dx = C.dropout_bwd(dy, mask, p, unit)
    assert rel_err(dx, torch.where(keep, dy.float() / (1 - p), torch.zeros_like(dy, dtype=torch.float32))) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,C,R,act,bias", [
    (128, 16, 96, 4, 2, True),       # EfficientNet-B0 stage-2 shapes
    (7, 2, 1152, 48, 2, True),       # last stage, ragged batch (< 8 samples per block)
    (33, 8, 512, 32, 1, True),       # SENet18 (ReLU)
    (70, 4, 440, 26, 1, False),      # RegNet-like, no bias, ragged tiles (C % 64, R odd)
    (1024, 4, 1152, 48, 2, True),    # bs1024: several sample chunks per channel tile
    (600, 2, 240, 10, 2, True),      # fused kernels: 2 samples per block
    (1030, 2, 96, 4, 1, False),      # fused kernels: 4 samples per block, ragged last block
])
def test_squeeze_excite_matches_fp32(N, H, C, R, act, bias):
    """Native squeeze-excite block (pool + fp32 MLP + sigmoid scale, and its backward with the
    parameter gradients added into given buffers) against the fp32 torch composition."""
    from pytorch_cifar_amd import _native

    L = _native.lib()
    assert L.se_supported(C, R)
    torch.manual_seed(0)
    x = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    w1 = torch.randn(R, C, 1, 1, device="cuda") * 0.1
    w2 = torch.randn(C, R, 1, 1, device="cuda") * 0.1
    b1 = torch.randn(R, device="cuda") if bias else None
    b2 = torch.randn(C, device="cuda") if bias else None
    out, pooled, hpre, s = L.se_forward(x, w1, b1, w2, b2, act)

    xr = x.float().requires_grad_(True)
    w1r, w2r = w1.clone().requires_grad_(True), w2.clone().requires_grad_(True)
    b1r = b1.clone().requires_grad_(True) if bias else None
    b2r = b2.clone().requires_grad_(True) if bias else None
    p = xr.mean((1, 2))
    h = torch.nn.functional.linear(p, w1r.view(R, C), b1r)
    h = torch.relu(h) if act == 1 else torch.nn.functional.silu(h)
    sr = torch.nn.functional.linear(h, w2r.view(C, R), b2r)
    ref = xr * torch.sigmoid(sr)[:, None, None, :]
    assert rel_err(pooled, p.detach()) < 1e-5
    assert rel_err(s, sr.detach()) < 1e-4
    assert rel_err(out, ref.detach()) < 1e-2

    dout = torch.randn_like(x)
    ref.backward(dout.float())
    dw10, dw20 = torch.randn(R * C, device="cuda"), torch.randn(R * C, device="cuda")
    db10, db20 = torch.randn(R, device="cuda"), torch.randn(C, device="cuda")
    acc = [t.clone() for t in (dw10, db10, dw20, db20)]
    dx, dw1, db1, dw2, db2 = L.se_backward(dout, x, pooled, hpre, s, w1, w2, act,
                                           acc[0], acc[1] if bias else None, acc[2],
                                           acc[3] if bias else None, bias, bias)
    assert dw1.data_ptr() == acc[0].data_ptr() and dw2.data_ptr() == acc[2].data_ptr()
    assert rel_err(dx, xr.grad) < 1e-2
    assert rel_err(dw1 - dw10, w1r.grad.view(-1)) < 1e-3
    assert rel_err(dw2 - dw20, w2r.grad.view(-1)) < 1e-3
    if bias:
        assert rel_err(db1 - db10, b1r.grad) < 1e-3
        assert rel_err(db2 - db20, b2r.grad) < 1e-3
    else:
        assert db1 is None and db2 is None


@pytest.mark.parametrize("N,H,Cin,Cout", [(8, 32, 64, 128), (16, 16, 128, 256), (32, 8, 256, 512),
                                          (2, 16, 128, 256)])
@pytest.mark.parametrize("cfg", [-1, 3, 7, 30])
def test_dgrad_compact_s2_addend(C, N, H, Cin, Cout, cfg):
    """Stride-2 dgrad with the projection shortcut's dX handed over compact ([N][H/2][W/2][Cin],
    even-even pixels): equal to the same kernel with the expanded addend, for the halo stride-2
    kernel, the parity igemm (split-K configs fall back to the expanded form) and the tuned choice;
    plus the fused BN-reduce form."""
    torch.manual_seed(11)
    Ho = H // 2
    dy = (torch.randn(N, Ho, Ho, Cout, device="cuda") * 0.5).bfloat16()
    w = torch.randn(Cout, 3, 3, Cin, device="cuda") * 0.05
    _, wt = C.weight_prep(w, 1, True)
    comp = torch.randn(N, Ho, Ho, Cin, device="cuda").bfloat16()
    full = torch.zeros(N, H, H, Cin, device="cuda").bfloat16()
    full[:, ::2, ::2, :] = comp
    C.set_conv_tile(0, cfg)
    try:
        ref = C.conv_dgrad(dy, wt, H, H, 2, 1, 1, full)
        got = C.conv_dgrad(dy, wt, H, H, 2, 1, 1, comp, True)
        assert torch.equal(got, ref)
        y = torch.randn(N, H, H, Cin, device="cuda").bfloat16()
        mask = torch.randint(0, 256, (y.numel() // 8,), device="cuda", dtype=torch.uint8)
        aux = torch.cat([torch.randn(Cin, device="cuda") * 0.1, torch.rand(Cin, device="cuda") + 0.5])
        r1, p1 = C.conv_dgrad_bn(dy, wt, H, H, 2, 1, 1, full, y, mask, aux)
        r2, p2 = C.conv_dgrad_bn(dy, wt, H, H, 2, 1, 1, comp, y, mask, aux, addend_s2c=True)
        assert torch.equal(r1, r2)
        if p1.numel():
            assert torch.allclose(p1.sum(0), p2.sum(0), rtol=1e-4, atol=1e-3)
    finally:
        C.set_conv_tile(0, -1)


@pytest.mark.parametrize("HW,Cc", [(32, 192), (16, 64), (8, 832), (4, 24)])
def test_maxpool3s1_rolling_ties(C, HW, Cc):
    """The rolling 3x3 / stride-1 / pad-1 max pool (csrc/pool.hip, GoogLeNet's Inception pool
    branch) on data full of ties: forward values exact, the gradient lands on the first maximum
    of each window in (kh, kw) order — where torch's fp32 max_pool2d puts it — and sums match."""
    torch.manual_seed(7)
    x = torch.randint(-3, 4, (3, Cc, HW, HW), device="cuda").float().requires_grad_(True)
    ref = F.max_pool2d(x, 3, 1, 1)
    dy = torch.randint(-4, 5, ref.shape, device="cuda").float()
    (g,) = torch.autograd.grad(ref, x, dy)
    xn = nhwc(x.detach()).bfloat16()
    y, arg = C.maxpool_fwd(xn, 3, 1, 1)
    assert torch.equal(nchw(y).float(), ref.detach())
    dx = C.maxpool_bwd(nhwc(dy).bfloat16(), arg, HW, HW, 3, 1, 1)
    assert torch.equal(nchw(dx).float(), g)     # small integers: every sum is exact in bf16


@pytest.mark.parametrize("k,HW,Cc", [(2, 32, 64), (2, 16, 456), (4, 8, 24), (8, 8, 1024)])
def test_avgpool_window_eq_stride(C, k, HW, Cc):
    """Vectorized k == s average pool (csrc/pool.hip: DenseNet transitions, pooled heads)."""
    torch.manual_seed(8)
    x = bf(torch.randn(4, Cc, HW, HW, device="cuda")).requires_grad_(True)
    ref = F.avg_pool2d(x.float(), k, k, 0)
    dy = bf(torch.randn_like(ref))
    (g,) = torch.autograd.grad(ref, x, dy)
    xn = nhwc(x.detach()).bfloat16()
    y = C.avgpool_fwd(xn, k, k, 0)
    assert rel_err(nchw(y), ref) < 4e-3
    dx = C.avgpool_bwd(nhwc(dy).bfloat16(), HW, HW, k, k, 0)
    assert rel_err(nchw(dx), g) < 4e-3


@pytest.mark.parametrize("case", [(8, 16, 96, 128, 32, -1), (8, 8, 256, 128, 64, -1),
                                  (4, 4, 512, 128, 128, 4)])
def test_dgrad_bn_fuse_row_strided_y(C, case):
    """The fused BatchNorm-backward reduce of a 1x1 dgrad reading a row-strided y (a DenseNet
    BatchNorm's input: a channel suffix of its block's concat slab, ops/functional.py DenseSlab):
    dX and the per-block sums are bitwise those of the same call on a dense copy of y (igemm and
    split-K forms), and the sums match fp32."""
    N, H, Cin, Cout, extra, split = case
    torch.manual_seed(11)
    slab = torch.randn(N, H, H, Cin + extra, device="cuda").to(torch.bfloat16)
    ys = slab[..., extra:]                       # row stride Cin + extra
    assert not ys.is_contiguous()
    yd = ys.contiguous()
    w = bf(torch.randn(Cout, Cin, 1, 1, device="cuda") * (1.0 / Cin) ** 0.5)
    _, wt = C.weight_prep(w.permute(0, 2, 3, 1).contiguous(), 1, True)
    dy = torch.randn(N, H, H, Cout, device="cuda").to(torch.bfloat16)
    mask_b = torch.rand(N, H, H, Cin, device="cuda") > 0.4
    bits = (mask_b.view(-1, 8).to(torch.int32) << torch.arange(8, device="cuda")).sum(1).to(torch.uint8)
    mean, istd = torch.randn(Cin, device="cuda") * 0.1, torch.rand(Cin, device="cuda") + 0.5
    aux = torch.cat([mean, istd])
    C.set_conv_tile(2, split)
    try:
        dx_d, p_d = C.conv_dgrad_bn(dy, wt, H, H, 1, 0, 1, None, yd, bits, aux)
        dx_s, p_s = C.conv_dgrad_bn(dy, wt, H, H, 1, 0, 1, None, ys, bits, aux)
    finally:
        C.set_conv_tile(2, -1)
    torch.cuda.synchronize()
    assert p_d.numel() > 0 and p_s.shape == p_d.shape
    assert torch.equal(dx_s, dx_d) and torch.equal(p_s, p_d)
    dz = torch.where(mask_b, dx_s.float(), torch.zeros_like(dx_s, dtype=torch.float32))
    s1 = dz.sum((0, 1, 2))
    s2 = (dz * (yd.float() - mean) * istd).sum((0, 1, 2))
    assert rel_err(p_s[:, 0, :].sum(0), s1) < 1e-3 and rel_err(p_s[:, 1, :].sum(0), s2) < 1e-3


@pytest.mark.parametrize("shape", [(8, 16, 32, 64, 96), (4, 8, 48, 256, 512)])
def test_bn_stats_copy_and_acc_view(C, shape):
    """DenseNet slab statistics cache: bn_stats_copy copies a tensor into its slab slice and adds
    its centred channel sums into a wider [R][2][ld] + K-row cache; bn_apply_acc reading a
    channel range of that cache (acc_off / acc_ld) gives the BatchNorm of the slab suffix —
    the copy bitwise, the output and running stats against fp32 batch statistics."""
    N, H, g, C0, Ctot = shape
    torch.manual_seed(5)
    R = 4
    cache = torch.empty(R * 2 * Ctot + Ctot, device="cuda")
    C.zero_(cache)
    slab = torch.zeros(N, H, H, Ctot, device="cuda", dtype=torch.bfloat16)
    x0 = (torch.randn(N, H, H, C0, device="cuda") * 3 + 20).to(torch.bfloat16)
    out = (torch.randn(N, H, H, g, device="cuda") * 0.5 - 4).to(torch.bfloat16)
    c0 = Ctot - C0
    C.bn_stats_copy(x0, slab[..., c0:], cache, c0, Ctot, R)
    c1 = c0 - g
    C.bn_stats_copy(out, slab[..., c1:c0], cache, c1, Ctot, R)
    torch.cuda.synchronize()
    assert torch.equal(slab[..., c0:], x0) and torch.equal(slab[..., c1:c0], out)
    y = slab[..., c1:]
    Cs = Ctot - c1
    yf = y.float().reshape(-1, Cs)
    gamma = torch.rand(Cs, device="cuda") + 0.5
    beta = torch.randn(Cs, device="cuda")
    rm, rv = torch.zeros(Cs, device="cuda"), torch.ones(Cs, device="cuda")
    nbt = torch.zeros(1, dtype=torch.long, device="cuda")
    o, mask, aux, _ = C.bn_apply_acc(y, cache, R, float(yf.shape[0]), gamma, beta, rm, rv, nbt, 0.1,
                                     1e-5, None, None, None, 0, None, None, None, None, None, 0.1,
                                     1e-5, 1, True, None, True, None, False, None, None,
                                     acc_off=c1, acc_ld=Ctot)
    m = yf.mean(0)
    v = yf.var(0, unbiased=False)
    ref = torch.relu((yf - m) / torch.sqrt(v + 1e-5) * gamma + beta)
    assert rel_err(aux[0], m) < 1e-5 and rel_err(aux[1], 1 / torch.sqrt(v + 1e-5)) < 1e-4
    assert rel_err(o.float().reshape(-1, Cs), ref) < 1e-2
    assert rel_err(rm, 0.1 * m) < 1e-5 and int(nbt.item()) == 1


@pytest.mark.parametrize("shape", [(8, 32, 16, 96), (4, 32, 24, 144), (9, 16, 32, 192),
                                   (4, 16, 40, 240), (3, 8, 24, 144), (2, 7, 16, 96),
                                   (8, 32, 144, 24), (4, 16, 96, 16), (2, 7, 240, 40),
                                   (3, 8, 256, 64), (4, 8, 72, 48)])
def test_conv1x1_narrow_k(C, shape):
    """Narrow-K 1x1 forward (csrc/conv1x1_nk.hip: the MobileNetV2 / EfficientNet expand convs,
    K <= 64, Cout = 96..240): output vs fp32 F.conv2d, BN statistics as slab rows (sum /
    sumsq of the stored bf16 values) and as shifted sums into a sharded accumulator + K row.
    (2, 7, 16, 96): 98 pixels, a partial 16-pixel group."""
    N, H, Cin, Cout = shape
    torch.manual_seed(3)
    x = bf(torch.randn(N, Cin, H, H, device="cuda"))
    w = bf(torch.randn(Cout, Cin, 1, 1, device="cuda") * (1.0 / Cin) ** 0.5)
    ref = F.conv2d(x, w)
    x_n = nhwc(x).to(torch.bfloat16)
    wb, _ = C.weight_prep(w.permute(0, 2, 3, 1).contiguous(), 1, False)
    prev = C.conv_nk_min_m(0)          # (production takes it from 512K pixels on)
    try:
        y, stats = C.conv_fwd(x_n, wb, None, 1, 0, 1, True)
        K = torch.randn(Cout, device="cuda")
        R = 4
        acc = torch.zeros(R * 2 * Cout + Cout, device="cuda")
        y2, _ = C.conv_fwd(x_n, wb, None, 1, 0, 1, True, acc, R, K)
    finally:
        C.conv_nk_min_m(prev)
    torch.cuda.synchronize()
    assert rel_err(nchw(y), ref) < 1e-2
    yf = y.float().reshape(-1, Cout)
    assert rel_err(stats[:, 0, :].sum(0), yf.sum(0)) < 1e-4
    assert rel_err(stats[:, 1, :].sum(0), (yf ** 2).sum(0)) < 1e-4
    assert torch.equal(y2, y)
    a = acc[:R * 2 * Cout].view(R, 2, Cout).sum(0)
    d = yf - K
    assert rel_err(a[0], d.sum(0)) < 1e-4 and rel_err(a[1], (d ** 2).sum(0)) < 1e-4
    assert torch.equal(acc[R * 2 * Cout:], K)


@pytest.mark.parametrize("shape", [(8, 32, 144, 24), (4, 16, 192, 32), (9, 16, 240, 40),
                                   (2, 7, 96, 16), (8, 32, 24, 144), (3, 8, 40, 240),
                                   (2, 7, 16, 96)])
def test_conv1x1_narrow_k_dgrad(C, shape):
    """Narrow-K kernel as the data gradient of a narrow-output 1x1 conv (the inverted-residual
    project conv: dX[M][Cin] = dY[M][Cout] . W^T, Cout <= 64): plain, and with the residual addend
    + fused BatchNorm-backward reduce (slab rows and sharded accumulator), vs fp32."""
    N, H, Cin, Cout = shape
    torch.manual_seed(4)
    w = bf(torch.randn(Cout, Cin, 1, 1, device="cuda") * (1.0 / Cin) ** 0.5)
    dy = bf(torch.randn(N, Cout, H, H, device="cuda"))
    ref = torch.nn.grad.conv2d_input((N, Cin, H, H), w, dy)
    _, wt = C.weight_prep(w.permute(0, 2, 3, 1).contiguous(), 1, True)
    dy_n = nhwc(dy).to(torch.bfloat16)
    ybn = torch.randn(N, H, H, Cin, device="cuda").to(torch.bfloat16)
    mask_b = torch.rand(N, H, H, Cin, device="cuda") > 0.4
    bits = (mask_b.view(-1, 8).to(torch.int32) << torch.arange(8, device="cuda")).sum(1).to(torch.uint8)
    mean, istd = torch.randn(Cin, device="cuda") * 0.1, torch.rand(Cin, device="cuda") + 0.5
    aux = torch.cat([mean, istd])
    add = torch.randn(N, H, H, Cin, device="cuda").to(torch.bfloat16)
    prev = C.conv_nk_min_m(0)
    try:
        dx = C.conv_dgrad(dy_n, wt, H, H, 1, 0, 1)
        dx2, part = C.conv_dgrad_bn(dy_n, wt, H, H, 1, 0, 1, add, ybn, bits, aux)
        R = 4
        bacc = torch.zeros(R * 2 * Cin, device="cuda")
        dx3, _ = C.conv_dgrad_bn(dy_n, wt, H, H, 1, 0, 1, add, ybn, bits, aux, bacc, R)
    finally:
        C.conv_nk_min_m(prev)
    torch.cuda.synchronize()
    assert rel_err(nchw(dx), ref) < 1e-2
    full = nhwc(ref) + add.float()
    assert rel_err(dx2, full) < 1e-2 and torch.equal(dx3, dx2)
    dz = torch.where(mask_b, dx2.float(), torch.zeros_like(full))
    s1 = dz.sum((0, 1, 2))
    s2 = (dz * (ybn.float() - mean) * istd).sum((0, 1, 2))
    assert part.numel() > 0
    assert rel_err(part[:, 0, :].sum(0), s1) < 1e-4 and rel_err(part[:, 1, :].sum(0), s2) < 1e-4
    a = bacc.view(R, 2, Cin).sum(0)
    assert rel_err(a[0], s1) < 1e-4 and rel_err(a[1], s2) < 1e-4


@pytest.mark.parametrize("N,R", [(128, 4), (1024, 4), (1000, 2)])
def test_fused_head_bn_backward_sums(N, R):
    """Head backward with the block-tail BatchNorm's backward sums (sum dz, sum dz * xhat of
    dz = dX * relu-mask) added into the [R][2][C] accumulator: the kernel gives each workgroup
    ceil(N / 64R) samples (<= 64 same-address atomics per shard row at any batch); sums against
    an fp32 torch reduction of the same dX, and dX itself against the plain head backward."""
    from pytorch_cifar_amd import _native

    C_ = _native.lib()
    torch.manual_seed(4)
    H, C, K = 4, 512, 10
    w = torch.randn(K, C, device="cuda") * 0.05
    pooled = torch.randn(N, C, device="cuda")
    dl = torch.randn(N, K, device="cuda")
    y = torch.randn(N, H, H, C, device="cuda").to(torch.bfloat16)
    bits = torch.randint(0, 2, (N * H * H * C,), device="cuda", dtype=torch.uint8)
    mask = (bits.view(-1, 8) << torch.arange(8, device="cuda", dtype=torch.uint8)).sum(1).to(torch.uint8)
    aux = torch.cat([torch.randn(C, device="cuda") * 0.1, torch.rand(C, device="cuda") + 0.5,
                     torch.zeros(2 * C, device="cuda")])
    acc = torch.zeros(R * 2 * C + C, device="cuda")
    dx, _, _ = C_.head_bwd(dl, w, pooled, H, H, None, None, True, 0.0, None, y, mask, aux, acc, R)
    dx0, _, _ = C_.head_bwd(dl, w, pooled, H, H, None, None, True)
    assert torch.equal(dx, dx0)
    dz = dx.float().view(N, H, H, C) * bits.view(N, H, H, C).float()
    xhat = (y.float() - aux[:C]) * aux[C:2 * C]
    s = acc[: R * 2 * C].view(R, 2, C).sum(0)
    assert rel_err(s[0], dz.sum((0, 1, 2))) < 1e-4
    assert rel_err(s[1], (dz * xhat).sum((0, 1, 2))) < 1e-4
