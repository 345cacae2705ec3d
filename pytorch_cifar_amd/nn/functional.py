"""Functional ops used by the model zoo (drop-in for the ``F.*`` calls of the reference models)."""
from ..ops.functional import (  # noqa: F401
    activation,
    adaptive_avg_pool2d,
    add_act,
    avg_pool2d,
    cat,
    channel_shuffle,
    cross_entropy,
    dropout,
    global_avg_pool,
    max_pool2d,
    relu,
    se_excite,
)


def swish(x):
    return activation(x, "swish")


def sigmoid(x):
    return activation(x, "sigmoid")


def se_gate(x, fc1, fc2, act="relu"):
    """Squeeze-and-excite: x * sigmoid(fc2(act(fc1(mean_hw(x))))).

    ``fc1``/``fc2`` are the reference's 1x1 ``Conv2d`` modules with bias (efficientnet.py:28-31,
    regnet.py:15-18, senet.py:59-60); on the pooled [N, C] vector they are plain GEMMs, so the
    squeeze runs on the native global-pool kernel, the two tiny FCs as library GEMMs in fp32 and
    the excitation (sigmoid + broadcast scale, and its backward) on the native SE kernel.
    """
    import torch.nn.functional as TF

    n, c = x.shape[0], x.shape[1]
    pooled = global_avg_pool(x).reshape(n, c).to(fc1.weight.dtype)
    h = TF.linear(pooled, fc1.weight.reshape(fc1.weight.shape[0], -1), fc1.bias)
    if act == "relu":
        h = TF.relu(h)
    elif act in ("swish", "silu"):
        h = h * h.sigmoid()
    s = TF.linear(h, fc2.weight.reshape(fc2.weight.shape[0], -1), fc2.bias)
    return se_excite(x, s)
