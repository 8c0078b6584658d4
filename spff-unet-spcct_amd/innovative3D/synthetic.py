"""Synthetic SPCCT batches (the reference's DICOM dataset is private and
offline).  Shapes follow the reference layouts: north-star ``[B, 5, D, H, W]``
(5 energy bins as channels) or registry ``[B, 1, 5, H, W]`` (bins on depth,
datasets.py:228-233).  Labels are int64 in [0, K) with a fraction set to
IGNORE_INDEX (255)."""
from __future__ import annotations

import torch


def synthetic_batch(batch=2, in_ch=5, depth=128, height=128, width=128, num_classes=13,
                    ignore_frac=0.01, seed=0, device="cpu"):
    g = torch.Generator(device="cpu").manual_seed(int(seed))
    x = torch.randn(batch, in_ch, depth, height, width, generator=g, dtype=torch.float32)
    y = torch.randint(0, num_classes, (batch, depth, height, width), generator=g, dtype=torch.int64)
    if ignore_frac > 0:
        m = torch.rand(batch, depth, height, width, generator=g) < ignore_frac
        y[m] = 255
    return x.to(device), y.to(device)


class SyntheticSPCCT(torch.utils.data.Dataset):
    """Map-style dataset of reproducible synthetic patches (one sample each)."""

    def __init__(self, n=8, in_ch=5, depth=128, height=128, width=128, num_classes=13, seed=0):
        self.n, self.shape, self.K, self.seed = n, (in_ch, depth, height, width), num_classes, seed

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        x, y = synthetic_batch(1, *self.shape, num_classes=self.K, seed=self.seed * 100003 + i)
        return x[0], y[0]
