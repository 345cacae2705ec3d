"""Small shared helpers for the model zoo."""
from __future__ import annotations


def shortcut_kwargs(shortcut, x):
    """Residual join arguments for ``BatchNorm2d.forward``.

    Identity shortcut -> ``residual=x``; projection shortcut ``Sequential(conv1x1, bn)`` ->
    ``residual_bn=(bn, conv(x))`` so both BatchNorms, the add and the ReLU run as one pass.
    """
    mods = list(shortcut)
    if not mods:
        return {"residual": x}
    if len(mods) == 2:
        conv, bn = mods
        return {"residual_bn": (bn, conv(x))}
    return {"residual": shortcut(x)}
