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
