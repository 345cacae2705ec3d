"""Functional ops used by the model zoo (drop-in for the ``F.*`` calls of the reference models)."""
import torch
import torch.nn.functional as TF

from ..engine import grads
from ..ops.functional import _ref
from ..ops.functional import (  # noqa: F401
    ChannelSlab,
    DenseSlab,
    activation,
    adaptive_avg_pool2d,
    add_act,
    avg_pool2d,
    bn_act_conv,
    bn_act_dwconv,
    cat,
    cat_shuffle2,
    cat_shuffle2_split,
    channel_shuffle,
    cross_entropy,
    dense_copy,
    dpn_merge,
    drop_connect,
    dropout,
    global_avg_pool,
    max_pool2d,
    pool_linear,
    relu,
    se_excite,
    split_channels,
    squeeze_excite,
)


def swish(x):
    return activation(x, "swish")


def sigmoid(x):
    return activation(x, "sigmoid")


class _SEMLP(torch.autograd.Function):
    """s = fc2(act(fc1(pooled))) on the pooled [N, C] fp32 vector, with the parameter gradients
    added straight into their gradient-arena views (``addmm_`` / ``addmv_`` with beta = 1) instead
    of autograd's separate mm + sum + AccumulateGrad add per parameter: ~4 launches fewer per SE
    block in backward (EfficientNet-B0 has 16)."""

    @staticmethod
    def forward(ctx, pooled, w1, b1, w2, b2, act):
        h_pre = torch.addmm(b1, pooled, w1.t()) if b1 is not None else pooled @ w1.t()
        h = torch.relu(h_pre) if act == "relu" else TF.silu(h_pre)
        s = torch.addmm(b2, h, w2.t()) if b2 is not None else h @ w2.t()
        ctx.save_for_backward(pooled, h_pre, h, w1, w2)
        ctx.act = act
        ctx.params = (w1, b1, w2, b2)
        return s

    @staticmethod
    def backward(ctx, ds):
        pooled, h_pre, h, w1, w2 = ctx.saved_tensors
        params = ctx.params
        ctx.params = None
        ds = ds.contiguous()
        out = [None, None, None, None]

        def deliver(i, p, a, b, vec):
            # p.grad += a^T b (weight) or a^T 1 (bias), in place in the arena when possible
            if p is None or not p.requires_grad:
                return
            base = getattr(p, "_pca_param", None)
            if base is not None and base.is_leaf:
                buf = grads.grad_buffer(base)
                if buf is not None:
                    buf = buf.reshape(-1)
                    if vec:
                        buf.addmv_(a.t(), _ones(a.shape[0], a.device))
                    else:
                        buf.view(a.shape[1], b.shape[1]).addmm_(a.t(), b)
                    grads.fire(base)
                    return
            out[i] = a.sum(0) if vec else a.t() @ b

        w1_, b1_, w2_, b2_ = params
        deliver(2, w2_, ds, h, False)
        deliver(3, b2_, ds, None, True)
        dh = ds @ w2
        dh_pre = (torch.ops.aten.threshold_backward(dh, h, 0) if ctx.act == "relu"
                  else torch.ops.aten.silu_backward(dh, h_pre))
        deliver(0, w1_, dh_pre, pooled, False)
        deliver(1, b1_, dh_pre, None, True)
        dpooled = dh_pre @ w1 if ctx.needs_input_grad[0] else None
        return dpooled, out[0], out[1], out[2], out[3], None


_ONES = {}


def _ones(n, device):
    key = (n, str(device))
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones(n, device=device)
    return t


def _mat(w):
    """[out, in, 1, 1] conv weight as a 2-D [out, in] view that remembers its parameter."""
    m = w.reshape(w.shape[0], -1)
    m._pca_param = w
    return m


def se_gate(x, fc1, fc2, act="relu"):
    """Squeeze-and-excite: x * sigmoid(fc2(act(fc1(mean_hw(x))))).

    ``fc1``/``fc2`` are the reference's 1x1 ``Conv2d`` modules with bias (efficientnet.py:28-31,
    regnet.py:15-18, senet.py:59-60); on the pooled [N, C] vector they are plain GEMMs, so the
    whole block normally runs as the native squeeze-excite kernels (pool, fp32 MLP, sigmoid scale;
    ``ops.functional.squeeze_excite``). Otherwise the squeeze runs on the native global-pool
    kernel, the two tiny FCs as library GEMMs in fp32 (:class:`_SEMLP` on the GPU, plain autograd
    on the CPU reference path) and the excitation on the native SE-scale kernel.
    """
    y = squeeze_excite(x, fc1.weight, fc1.bias, fc2.weight, fc2.bias, act)
    if y is not None:
        return y
    n, c = x.shape[0], x.shape[1]
    pooled = global_avg_pool(x).reshape(n, c).to(fc1.weight.dtype)
    if (not _ref(x) and act in ("relu", "swish", "silu") and pooled.dtype == torch.float32
            and not torch.is_autocast_enabled()):
        b1 = fc1.bias
        b2 = fc2.bias
        if b1 is not None:
            b1._pca_param = b1
        if b2 is not None:
            b2._pca_param = b2
        s = _SEMLP.apply(pooled, _mat(fc1.weight), b1, _mat(fc2.weight), b2,
                         "relu" if act == "relu" else "silu")
        return se_excite(x, s)
    h = TF.linear(pooled, fc1.weight.reshape(fc1.weight.shape[0], -1), fc1.bias)
    if act == "relu":
        h = TF.relu(h)
    elif act in ("swish", "silu"):
        h = h * h.sigmoid()
    s = TF.linear(h, fc2.weight.reshape(fc2.weight.shape[0], -1), fc2.bias)
    return se_excite(x, s)
