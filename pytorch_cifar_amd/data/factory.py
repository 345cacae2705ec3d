"""Dataset + loader construction shared by main.py / main_dist.py / bench.py."""
from __future__ import annotations

from .cifar10 import load_cifar10
from .loader import DeviceLoader
from .synthetic import synthetic_cifar10


def load_split(data_dir, train, synthetic=False, synthetic_size=None, seed=0):
    if synthetic:
        n = synthetic_size or (50000 if train else 10000)
        return synthetic_cifar10(n, seed=seed + (0 if train else 1))
    return load_cifar10(data_dir, train=train)


def build_loaders(data_dir="./data", synthetic=False, batch_size=128, test_batch_size=100,
                  device="cpu", world=1, rank=0, crop_pad=4, flip=True, seed=0,
                  synthetic_size=None, test_synthetic_size=None):
    tr_x, tr_y = load_split(data_dir, True, synthetic, synthetic_size, seed)
    te_x, te_y = load_split(data_dir, False, synthetic, test_synthetic_size, seed)
    train = DeviceLoader(tr_x, tr_y, batch_size, device, train=True, shuffle=True, crop_pad=crop_pad,
                         flip=flip, world=world, rank=rank, seed=seed)
    test = DeviceLoader(te_x, te_y, test_batch_size, device, train=False, shuffle=False,
                        world=world, rank=rank, seed=seed)
    return train, test
