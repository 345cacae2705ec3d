"""GPU-resident CIFAR input pipeline (replaces torchvision transforms + DataLoader workers).

Reference pipeline (main.py:30-50, main_dist.py:93-132): PIL RandomCrop(32, padding=4) ->
RandomHorizontalFlip -> ToTensor -> Normalize(mean, std) in CPU worker processes, then an H2D
copy per batch.  Here the whole uint8 dataset (150 MB) lives in HBM and one
augmentation kernel per batch gathers the sampled images, applies crop/flip/normalize and writes
the bf16 NHWC tensor the first conv consumes (RGB padded to 8 channels).  No host work or H2D
traffic per step, and the augmentation is capturable into the training step's hipGraph.

Training shards follow ``torch.utils.data.DistributedSampler`` exactly (seed + epoch permutation,
padding to a multiple of the world size, ``indices[rank::world]``), with ``set_epoch`` honoured
(the reference never calls it, main_dist.py:110 — SURVEY App. B #7). Evaluation shards are not
padded, so the all-reduced test accuracy counts each of the 10,000 images exactly once (the
reference evaluated the full set on every rank, main_dist.py:129-132).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import _native
from ..ops.functional import padded_input
from .cifar10 import MEAN, STD


class ShardSampler:
    """DistributedSampler-equivalent index generator (CPU-side, once per epoch)."""

    def __init__(self, n, world=1, rank=0, shuffle=True, seed=0, drop_last=False, pad=True):
        self.n, self.world, self.rank = n, world, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        # pad=False (evaluation): no duplicated samples, ranks differ by at most one sample and the
        # all-reduced counts cover the dataset exactly once
        self.pad = pad
        self.epoch = 0
        if not pad:
            self.num_samples = len(range(rank, n, world))
        elif drop_last and n % world:
            self.num_samples = math.ceil((n - world) / world)
        else:
            self.num_samples = math.ceil(n / world)
        self.total_size = self.num_samples * world

    def set_epoch(self, epoch):
        self.epoch = epoch

    def indices(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g)
        else:
            idx = torch.arange(self.n)
        if not self.pad:
            return idx[self.rank::self.world]
        if not self.drop_last:
            pad = self.total_size - idx.numel()
            if pad > 0:
                reps = math.ceil(pad / idx.numel())
                idx = torch.cat([idx, idx.repeat(reps)[:pad]])
        else:
            idx = idx[: self.total_size]
        return idx[self.rank: self.total_size: self.world]

    def __len__(self):
        return self.num_samples


class DeviceLoader:
    """Iterates (inputs, targets) batches produced on-device.

    ``crop_pad`` 4 + ``flip`` reproduces main.py's train transform; ``crop_pad`` 0 + ``flip`` is
    main_dist.py's; both 0 is the test transform. On CPU the same transforms run in torch.
    """

    def __init__(self, images: np.ndarray, labels: np.ndarray, batch_size: int, device,
                 train=True, shuffle=True, crop_pad=4, flip=True, world=1, rank=0, seed=0,
                 drop_last=False, mean=MEAN, std=STD):
        self.device = torch.device(device)
        self.batch_size = batch_size
        self.train = train
        self.crop_pad = crop_pad if train else 0
        self.flip = flip if train else False
        self.fp32 = False
        self.mean, self.std = tuple(mean), tuple(std)
        self.drop_last = drop_last
        self.sampler = ShardSampler(len(labels), world, rank, shuffle, seed, drop_last=False,
                                    pad=train)
        self.images = torch.from_numpy(np.ascontiguousarray(images)).to(self.device)
        self.labels = torch.from_numpy(np.asarray(labels, dtype=np.int64)).to(self.device)
        self.gen = torch.Generator(device="cpu")
        self.gen.manual_seed(seed * 1000003 + rank)
        self._idx = None

    def set_epoch(self, epoch: int):
        self.sampler.set_epoch(epoch)

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def epoch_indices(self) -> torch.Tensor:
        return self.sampler.indices().to(self.device)

    @property
    def packed(self) -> bool:
        """GPU loaders hand out packed batch entries ``sample | word << 32``: the epoch's
        augmentation words are drawn in one launch at epoch start, so a (graph-captured) training
        step needs no RNG or label-gather launches — one augment kernel makes images + targets."""
        return self.device.type == "cuda"

    def batch_indices(self):
        """Per-batch device tensors of the epoch (packed entries on GPU, see :attr:`packed`)."""
        idx = self.epoch_indices()
        if self.packed:
            idx = idx | (self.random_words(idx.numel()).to(torch.int64) << 32)
        for b in range(len(self)):
            yield idx[b * self.batch_size: (b + 1) * self.batch_size]

    @staticmethod
    def sample_ids(batch: torch.Tensor) -> torch.Tensor:
        """Dataset indices of a batch from :meth:`batch_indices` (packed or not)."""
        return batch & 0xFFFFFFFF

    def random_words(self, n: int) -> torch.Tensor:
        """Per-sample augmentation word k (int32), uniform over every (dy, dx, flip) triple:
        dy = k % span, dx = (k // span) % span, flip = k // span**2 with span = 2 * crop_pad + 1
        (torchvision RandomCrop / RandomHorizontalFlip draw each offset and the flip uniformly)."""
        p = self.crop_pad
        span = 2 * p + 1
        if not self.train or (p == 0 and not self.flip):
            return torch.full((n,), p + p * span, dtype=torch.int32, device=self.device)
        # GPU: the default generator (seeded by torch.manual_seed), drawn once per epoch
        gen = None if self.device.type == "cuda" else self.gen
        hi = span * span * (2 if self.flip else 1)
        return torch.randint(0, hi, (n,), generator=gen, device=self.device, dtype=torch.int32)

    def make_batch(self, idx: torch.Tensor, rnd: torch.Tensor | None = None):
        """Gather + augment the samples ``idx`` -> (NCHW-shaped inputs, int64 targets).

        On GPU ``idx`` holds packed entries from :meth:`batch_indices` (unless ``rnd`` is given)."""
        if self.device.type == "cuda" and rnd is None:
            out, targets = _native.lib().augment_packed(self.images, self.labels, idx, self.crop_pad,
                                                        list(self.mean), list(self.std))
            x = padded_input(out, 3)
            if self.fp32:
                x = x.float()
            return x, targets
        if rnd is None:
            rnd = self.random_words(idx.numel())
        targets = self.labels.index_select(0, idx)
        if self.device.type == "cuda":
            out = _native.lib().augment(self.images, idx, rnd, self.crop_pad, list(self.mean), list(self.std))
            x = padded_input(out, 3)
            if self.fp32:   # --dtype fp32: stock fp32 kernels consume an fp32 channels_last batch
                x = x.float()
            return x, targets
        return self._cpu_batch(idx, rnd), targets

    def _cpu_batch(self, idx, rnd):
        x = self.images.index_select(0, idx).permute(0, 3, 1, 2).float().div_(255.0)
        p = self.crop_pad
        n = x.shape[0]
        if p:
            H, W = x.shape[2], x.shape[3]
            xp = torch.nn.functional.pad(x, (p, p, p, p))
            dy = (rnd % (2 * p + 1)).long()
            dx = ((rnd // (2 * p + 1)) % (2 * p + 1)).long()
            rows = (dy[:, None] + torch.arange(H)).view(n, 1, H, 1).expand(n, 3, H, W + 2 * p)
            xr = xp.gather(2, rows)
            cols = (dx[:, None] + torch.arange(W)).view(n, 1, 1, W).expand(n, 3, H, W)
            x = xr.gather(3, cols)
        if self.flip:
            f = ((rnd // ((2 * p + 1) ** 2)) & 1).bool()
            x[f] = x[f].flip(3)
        m = torch.tensor(self.mean).view(1, 3, 1, 1)
        s = torch.tensor(self.std).view(1, 3, 1, 1)
        return (x - m) / s

    def __iter__(self):
        for idx in self.batch_indices():
            if self.drop_last and idx.numel() < self.batch_size:
                break
            yield self.make_batch(idx)
