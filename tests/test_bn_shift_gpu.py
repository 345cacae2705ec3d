"""Shifted BatchNorm forward sums at the producer kernels (csrc/common.h stat_shift): for every
forward kernel family that delivers statistics (stem, layer-1 c64, halo hx, generic igemm, 1x1,
split-K reduce), in slab and sharded-accumulator form:

* the conv output does not depend on the shift (bitwise);
* a zero shift gives bitwise the unshifted sums;
* a shift K gives sums of (x - K) (against fp64 on the bf16 output) and, in accumulator form,
  publishes K in the accumulator's K row.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

# (N, Cin, H, Cout, k, stride, pad, cfg): cfg = forced tile config (-1: default selection)
CASES = [
    (64, 8, 32, 64, 3, 1, 1, -1),       # stem kernel (8-channel padded RGB)
    (64, 64, 32, 64, 3, 1, 1, -1),      # layer-1 c64
    (64, 128, 16, 128, 3, 1, 1, 30),    # halo hx
    (64, 512, 4, 512, 3, 1, 1, 3),      # generic igemm
    (64, 96, 8, 576, 1, 1, 0, 3),       # 1x1 (MobileNetV2 expand)
    (16, 256, 4, 256, 3, 1, 1, 3),      # small M: split-K candidate
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("acc_form", [False, True])
@pytest.mark.parametrize("det", [False, True])
def test_shifted_stats(case, acc_form, det):
    import pytorch_cifar_amd
    from pytorch_cifar_amd import _native

    C = _native.lib()
    N, Cin, H, Cout, k, s, p, cfg = case
    torch.manual_seed(0)
    x = (torch.randn(N, H, H, Cin, device="cuda") + 3.0).bfloat16()
    w = torch.randn(Cout, k, k, Cin, device="cuda") * (2.0 / (Cin * k * k)) ** 0.5
    wb, _ = C.weight_prep(w, 1, False)
    R = 8

    def run(shift):
        if acc_form:
            acc = torch.zeros(R * 2 * Cout + Cout, device="cuda")
            y, _ = C.conv_fwd(x, wb, None, s, p, 1, True, acc, R, shift)
            sums = acc[: R * 2 * Cout].view(R, 2, Cout).sum(0)
            return y, sums, acc[R * 2 * Cout:]
        y, st = C.conv_fwd(x, wb, None, s, p, 1, True, None, 0, shift)
        return y, st.sum(0), None

    C.set_conv_tile(0, cfg)
    C.set_conv_tile(2, 3 if case[0] == 16 else -1)
    pytorch_cifar_amd.set_deterministic(det)
    try:
        y0, s0, _ = run(None)
        yz, sz, kz = run(torch.zeros(Cout, device="cuda"))
        K = torch.randn(Cout, device="cuda") + 3.0
        yk, sk, kk = run(K)
    finally:
        pytorch_cifar_amd.set_deterministic(False)
        C.set_conv_tile(0, -1)
        C.set_conv_tile(2, -1)
    assert torch.equal(y0, yz) and torch.equal(y0, yk), "the shift must not change the output"
    if not acc_form:   # (atomic accumulation order varies between launches)
        assert torch.equal(s0, sz), "a zero shift must give the unshifted sums bitwise"
    else:
        torch.testing.assert_close(sz, s0, rtol=1e-5, atol=1e-2)
        assert torch.equal(kk, K), "the accumulator's K row must hold the shift"
    # the kernels sum the fp32 accumulators, the oracle sums the bf16-rounded outputs (<= 2^-8
    # relative per element): bound by that rounding plus fp32 summation; a wrong or missing shift
    # is off by ~K per term, i.e. by n*K
    d = yk.double().reshape(-1, Cout) - K.double()
    ya = yk.double().reshape(-1, Cout).abs()
    tol1 = ya.sum(0) / 256 + 1e-4 * d.abs().sum(0) + 1e-2
    tol2 = (2 * d.abs() * ya).sum(0) / 256 + 1e-4 * (d * d).sum(0) + 1e-2
    assert ((sk[0].double() - d.sum(0)).abs() <= tol1).all()
    assert ((sk[1].double() - (d * d).sum(0)).abs() <= tol2).all()


def test_one_conv_output_two_bns_slab_path(monkeypatch):
    """on the slab path a conv's sums carry a snapshot of the shift K they
    were taken against, so two BNs finalizing the same conv output one after the other (the second
    reading sums whose live pilot the first finalize has already overwritten) both get the right
    batch mean / running mean. Accumulators disabled; three steps so the pilot is non-zero."""
    import torch.nn.functional as TF

    from pytorch_cifar_amd.nn import BatchNorm2d, Conv2d
    from pytorch_cifar_amd.ops import functional as OF

    monkeypatch.setattr(OF, "acc_enabled", lambda *a, **k: False)
    torch.manual_seed(4)
    conv = Conv2d(32, 64, 3, padding=1, bias=False).cuda()
    bn_a, bn_b = BatchNorm2d(64).cuda(), BatchNorm2d(64).cuda()
    ref_rm = torch.zeros(64, device="cuda")
    ref_rv = torch.ones(64, device="cuda")
    for step in range(3):
        x = (torch.randn(16, 32, 8, 8, device="cuda") + 3.0).bfloat16().contiguous(memory_format=torch.channels_last)
        with torch.no_grad():
            y = conv(x)
            a = bn_a(y, act="relu")
            b = bn_b(y)
            yf = y.float()
            ref = TF.batch_norm(yf, ref_rm, ref_rv, None, None, True, 0.1, 1e-5)
        assert (b.float() - ref).abs().max() < 5e-2, step
        assert (a.float() - ref.clamp_min(0)).abs().max() < 5e-2, step
    for bn in (bn_a, bn_b):
        assert torch.allclose(bn.running_mean, ref_rm, rtol=1e-3, atol=1e-3)
        assert torch.allclose(bn.running_var, ref_rv, rtol=1e-2, atol=1e-3)
