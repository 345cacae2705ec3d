"""Synthetic CIFAR-shaped data (no dataset files / network in the benchmark environment)."""
from __future__ import annotations

import numpy as np


def synthetic_cifar10(n: int = 50000, seed: int = 0, num_classes: int = 10):
    """uint8 images [n, 32, 32, 3] + int64 labels [n], deterministic for a seed.

    Labels are a weak function of the image's mean colour so a few training steps move the loss
    (useful for smoke tests), but nothing here is meant to be learnable in earnest.
    """
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, num_classes, size=n, dtype=np.int64)
    base = rng.integers(0, 256, size=(n, 32, 32, 3), dtype=np.uint8)
    tint = (labels * (255 // num_classes)).astype(np.uint8)
    base[:, :4, :4, 0] = tint[:, None, None]
    return base, labels
