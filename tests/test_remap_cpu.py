"""Host-side checks of the channel-remap maps (group pad / unpad / shuffle / weight pad) that the
native ``chan_remap`` kernel consumes: each map applied with torch indexing reproduces the stock
op, and the inverse map is the adjoint (the backward the kernel runs)."""
import torch

from pytorch_cifar_amd.ops import functional as OF


def _apply(x, cmap, rmap=None, K=1):
    """torch emulation of chan_remap: x [rows, Cin] -> [Q, J], -1 entries give zeros."""
    cm = torch.tensor(cmap)
    xz = torch.cat([x, torch.zeros(x.shape[0], 1, dtype=x.dtype)], 1)   # column -1 -> zero
    out = xz[:, torch.where(cm < 0, x.shape[1], cm)]
    if rmap is None:
        return out
    rows = out.view(-1, K, out.shape[1])
    rows = torch.cat([rows, torch.zeros(1, K, out.shape[1], dtype=x.dtype)], 0)
    rm = torch.tensor(rmap)
    return rows[torch.where(rm < 0, rows.shape[0] - 1, rm)].reshape(-1, out.shape[1])


def _adjoint_ok(remap, rows_in, K=1):
    x = torch.randn(rows_in, remap.cin, dtype=torch.float64)
    y = _apply(x, remap.cmap, remap.rmap, K)
    g = torch.randn_like(y)
    back = _apply(g, remap.icmap, remap.irmap, K)
    assert torch.allclose((y * g).sum(), (x * back).sum())


def test_group_pad_unpad_maps():
    G, n, npad = 3, 25, 32
    pad = OF._group_pad_remap(G, n, npad)
    unpad = OF._group_unpad_remap(G, n, npad)
    x = torch.randn(10, G * n)
    xp = _apply(x, pad.cmap)
    ref = torch.nn.functional.pad(x.view(10, G, n), (0, npad - n)).reshape(10, G * npad)
    assert torch.equal(xp, ref)
    assert torch.equal(_apply(xp, unpad.cmap), x)
    _adjoint_ok(pad, 7)
    _adjoint_ok(unpad, 7)


def test_shuffle_map():
    for C, g in [(200, 2), (240, 3), (30, 3)]:
        sh = OF._shuffle_remap(C, g)
        x = torch.randn(4, C)
        ref = x.view(4, g, C // g).transpose(1, 2).reshape(4, C)
        assert torch.equal(_apply(x, sh.cmap), ref)
        _adjoint_ok(sh, 4)


def test_weight_pad_map():
    G, cout_g, op, Cg, cp, K = 2, 25, 32, 13, 16, 9
    wr = OF._weight_pad_remap(G, cout_g, op, Cg, cp, K)
    w = torch.randn(G * cout_g, K, Cg)
    out = _apply(w.reshape(-1, Cg), wr.cmap, wr.rmap, K).view(G * op, K, cp)
    ref = torch.nn.functional.pad(w.view(G, cout_g, K, Cg), (0, cp - Cg, 0, 0, 0, op - cout_g))
    assert torch.equal(out, ref.reshape(G * op, K, cp))
    _adjoint_ok(wr, G * cout_g * K, K)
