"""CIFAR-10 without torchvision (reference main.py:41-50 uses torchvision.datasets.CIFAR10).

Reads either on-disk format into one uint8 [N, 32, 32, 3] array (NHWC, RGB) + int64 labels:

* ``cifar-10-batches-bin``  — the binary release: records of 1 label byte + 3072 pixel bytes
  (R plane, G plane, B plane). Parsed with numpy, no code execution from the file.
* ``cifar-10-batches-py``   — the python release (pickled dicts). Unpickled with a restricted
  unpickler that only admits the numpy/builtin types the release contains.

There is no network in this environment: ``download=True`` raises a clear error instead of
fetching. Use :mod:`pytorch_cifar_amd.data.synthetic` for shape-identical synthetic data.
"""
from __future__ import annotations

import io
import os
import pickle

import numpy as np

MEAN = (0.4914, 0.4822, 0.4465)  # main.py:34
STD = (0.2023, 0.1994, 0.2010)
CLASSES = ("plane", "car", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck")

_BIN_TRAIN = [f"data_batch_{i}.bin" for i in range(1, 6)]
_BIN_TEST = ["test_batch.bin"]
_PY_TRAIN = [f"data_batch_{i}" for i in range(1, 6)]
_PY_TEST = ["test_batch"]


def _read_bin(paths):
    imgs, labels = [], []
    for p in paths:
        raw = np.fromfile(p, dtype=np.uint8)
        if raw.size % 3073:
            raise ValueError(f"{p}: not a CIFAR-10 binary batch")
        rec = raw.reshape(-1, 3073)
        labels.append(rec[:, 0].astype(np.int64))
        imgs.append(rec[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1))
    return np.ascontiguousarray(np.concatenate(imgs)), np.concatenate(labels)


class _SafeUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"),
        ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"),
        ("numpy", "dtype"),
        ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"),
        ("builtins", "bytes"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a dataset file")


def _read_py(paths):
    imgs, labels = [], []
    for p in paths:
        with open(p, "rb") as f:
            d = _SafeUnpickler(io.BytesIO(f.read()), encoding="latin1").load()
        data = d.get("data", d.get(b"data"))
        lab = d.get("labels", d.get(b"labels"))
        imgs.append(np.asarray(data, dtype=np.uint8).reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1))
        labels.append(np.asarray(lab, dtype=np.int64))
    return np.ascontiguousarray(np.concatenate(imgs)), np.concatenate(labels)


def find_root(root: str):
    for sub, kind in (("cifar-10-batches-bin", "bin"), ("cifar-10-batches-py", "py")):
        d = os.path.join(root, sub)
        if os.path.isdir(d):
            return d, kind
    return None, None


def load_cifar10(root: str = "./data", train: bool = True, download: bool = False):
    """Return (images uint8 [N,32,32,3], labels int64 [N])."""
    d, kind = find_root(root)
    if d is None:
        msg = (f"CIFAR-10 not found under {root!r} (expected cifar-10-batches-bin/ or "
               "cifar-10-batches-py/).")
        if download:
            msg += " Downloading is not possible in this environment (no network)."
        raise FileNotFoundError(msg + " Use --synthetic for shape-identical synthetic data.")
    if kind == "bin":
        names = _BIN_TRAIN if train else _BIN_TEST
        return _read_bin([os.path.join(d, n) for n in names])
    names = _PY_TRAIN if train else _PY_TEST
    return _read_py([os.path.join(d, n) for n in names])


def get_mean_and_std(images: np.ndarray):
    """Per-channel mean/std (utils.py:16-28 semantics: mean over per-image statistics)."""
    x = images.astype(np.float32) / 255.0
    per_img_mean = x.mean(axis=(1, 2))
    per_img_std = x.std(axis=(1, 2), ddof=1)
    return per_img_mean.mean(0), per_img_std.mean(0)
