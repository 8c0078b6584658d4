"""Training data path (mirror of innovative3D/datasets.py + the volume builder of
helpers.py), device-resident.  SURVEY §8(f) rank 4.

The reference decodes DICOM stacks on the host, resizes each frame with
``TF.resize``, rasterises the ellipse ROIs in a pure-Python pixel loop
(helpers.py:132-211), keeps the volumes as host numpy arrays and augments every
sample in DataLoader worker processes (``TrainGridAug``, datasets.py:131-209).
Here the volumes live in HBM (a 512 x 512 x 5 volume is 5 MB; hundreds fit in
288 GB), the resize / rasterisation / augmentation run as HIP kernels
(csrc/data.hip), and a batch is assembled on the device with no worker
processes.  The random decisions keep the reference's exact draw order on
Python's module-level ``random`` (so ``random.seed`` reproduces the reference's
decisions); only the gaussian-noise values come from a counter-based device RNG
instead of ``torch.randn_like``.  The shuffled sample order is RandomSampler's
(torch default generator), as the reference DataLoader draws it.  One stated
difference: the reference augments in 16 worker processes, each re-seeding
``random`` per worker, so its per-sample decisions are reproducible only with
num_workers=0; that single-process order is the one kept here.

DICOM decoding: ``read_dicom_frames`` uses pydicom when it is installed and otherwise the
native reader of innovative3D/dicom.py (uncompressed transfer syntaxes).
"""
from __future__ import annotations

import os
import random
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _engine as E
from .config import IGNORE_INDEX, NUM_CLASSES

__all__ = ["_grid_boundaries", "_shuffle_stripes", "TrainGridAug", "DicomDataset3D",
           "DeviceBatchLoader", "MultiDicomDataModule3D", "stripe_maps"]


def _grid_boundaries(n: int, g: int):
    """datasets.py:56-58 (ragged edges allowed)."""
    return [(i * n) // g for i in range(g)] + [n]


def _axis_map(n: int, g: int, rng) -> List[int]:
    src = list(range(n))
    b = _grid_boundaries(n, max(1, int(g)))
    groups = {}
    for i in range(len(b) - 1):
        groups.setdefault(b[i + 1] - b[i], []).append((b[i], b[i + 1]))
    for _size, lst in groups.items():
        perm = lst[:]
        rng.shuffle(perm)
        for (t0, t1), (s0, _s1) in zip(lst, perm):
            src[t0:t1] = range(s0, s0 + (t1 - t0))
    return src


def stripe_maps(H: int, W: int, g_rows: int, g_cols: int, rng=random):
    """The separable stripe shuffle of datasets.py:60-115 as (row_src, col_src):
    stripes swap only with stripes of the same size; rows are drawn before columns."""
    if g_rows <= 1 and g_cols <= 1:
        return list(range(H)), list(range(W))
    return _axis_map(H, g_rows, rng), _axis_map(W, g_cols, rng)


def _shuffle_stripes(x: torch.Tensor, y: Optional[torch.Tensor], g_rows: int, g_cols: int):
    """datasets.py:60-115 on the device: one gather through the drawn maps."""
    rs, cs = stripe_maps(x.shape[-2], x.shape[-1], g_rows, g_cols)
    rs = torch.as_tensor(rs, device=x.device)
    cs = torch.as_tensor(cs, device=x.device)
    xo = x.index_select(-2, rs).index_select(-1, cs)
    yo = None if y is None else y.index_select(-2, rs).index_select(-1, cs)
    return xo, yo


class TrainGridAug:
    """datasets.py:131-209: flips, rot90, jitter, noise, per-sample grid shuffle and
    the top-left stamp -- decisions drawn on the host in the reference's order,
    applied by one fused device kernel (spff_grid_aug)."""

    def __init__(self, gs_choices=(2, 3, 4, 5), p_grid=1.0, flip_p=0.5, rot90_p=0.5,
                 jitter_p=0.3, noise_p=0.3, noise_std=0.01, stamp_top_left=True):
        self.gs_choices = tuple(int(g) for g in gs_choices)
        self.p_grid = float(p_grid)
        self.flip_p = float(flip_p)
        self.rot90_p = float(rot90_p)
        self.jitter_p = float(jitter_p)
        self.noise_p = float(noise_p)
        self.noise_std = float(noise_std)
        self.stamp = bool(stamp_top_left)

    def draw(self, H: int, W: int, gs: Optional[int], rng=random):
        """-> (prm[8], row_src, col_src, (Ho, Wo)) for one sample."""
        fw = rng.random() < self.flip_p
        fh = rng.random() < self.flip_p
        rot = rng.randint(1, 3) if rng.random() < self.rot90_p else 0
        jit, scale, shift = 0.0, 1.0, 0.0
        if rng.random() < self.jitter_p:
            jit = 1.0
            scale = 1.0 + 0.1 * (2 * rng.random() - 1)
            shift = 0.05 * (2 * rng.random() - 1)
        noise = rng.random() < self.noise_p
        run_grid = rng.random() < self.p_grid
        use_gs = int(gs) if gs is not None else None
        if use_gs is None or use_gs < 1:
            use_gs = rng.choice(self.gs_choices) if self.gs_choices else 1
        Ho, Wo = (W, H) if rot % 2 else (H, W)
        grid = run_grid and use_gs > 1
        rs, cs = stripe_maps(Ho, Wo, use_gs, use_gs, rng) if grid else (list(range(Ho)),
                                                                       list(range(Wo)))
        prm = [float(fw), float(fh), float(rot), jit, scale, shift,
               self.noise_std if noise else 0.0, float(grid and self.stamp)]
        return prm, rs, cs, (Ho, Wo)

    def __call__(self, x: torch.Tensor, y: Optional[torch.Tensor], gs: Optional[int]):
        """x: (1,F,H,W) device volume, y: (F,H,W) or None (the reference's 3D layout)."""
        assert x.ndim == 4 and x.shape[0] == 1, f"expected (1,F,H,W), got {tuple(x.shape)}"
        xo, yo = self.batch(x, None if y is None else y.unsqueeze(0), [gs])
        return xo, (None if yo is None else yo[0])

    def batch(self, x: torch.Tensor, y: Optional[torch.Tensor], gss: Sequence[Optional[int]],
              seed: Optional[int] = None):
        """x [B,F,H,W] (+ y [B,F,H,W]) -> augmented batch.  With H != W every sample of one
        call must share the rot90 parity (same output shape); H == W always works."""
        B, F_, H, W = x.shape
        draws = [self.draw(H, W, g) for g in gss]
        shapes = {d[3] for d in draws}
        if len(shapes) != 1:
            raise ValueError("samples of one batch rotate to different shapes (H != W)")
        maps = torch.tensor([d[1] + d[2] for d in draws], dtype=torch.int32)
        prm = torch.tensor([d[0] for d in draws], dtype=torch.float32)
        if seed is None:
            seed = random.getrandbits(63)
        return E.grid_aug(x.float(), y, maps.to(x.device, non_blocking=True),
                          prm.to(x.device, non_blocking=True), seed, shapes.pop())


class DicomDataset3D(torch.utils.data.Dataset):
    """datasets.py:212-238 over device-resident volumes: images [N,F,H,W],
    labels [N,F,H,W]; labels >= NUM_CLASSES become IGNORE_INDEX; a sample is
    ((1,F,H,W) image, (F,H,W) labels) after the transform."""

    def __init__(self, images, labels, grid_sizes, transform=None, device=None):
        dev = device or (torch.device("cuda") if torch.cuda.is_available() else None)
        self.images = torch.as_tensor(images, dtype=torch.float32, device=dev)
        lab = torch.as_tensor(labels, dtype=torch.int64, device=dev)
        self.labels = torch.where(lab >= NUM_CLASSES, torch.full_like(lab, IGNORE_INDEX), lab)
        self.grid_sizes = list(int(g) for g in grid_sizes)
        self.transform = transform

    def __len__(self):
        return int(self.images.shape[0])

    def __getitem__(self, idx):
        img = self.images[idx].unsqueeze(0)
        lbl = self.labels[idx]
        if self.transform:
            img, lbl = self.transform(img, lbl, self.grid_sizes[idx])
        return img, lbl


class DeviceBatchLoader:
    """The DataLoader of datasets.py:318-338 without worker processes: shuffled
    index batches gathered from the HBM-resident dataset and augmented as one
    batch (one fused kernel launch)."""

    def __init__(self, ds: DicomDataset3D, batch_size: int, shuffle: bool, drop_last=False):
        self.ds, self.bs, self.shuffle, self.drop_last = ds, int(batch_size), shuffle, drop_last

    def __len__(self):
        n = len(self.ds)
        return n // self.bs if self.drop_last else (n + self.bs - 1) // self.bs

    def __iter__(self):
        # torch's default-generator draws in DataLoader order: the iterator's base
        # seed (dataloader.py _BaseDataLoaderIter.__init__), then RandomSampler's
        # shuffle seed and its randperm (sampler.py RandomSampler.__iter__) -- so a
        # seeded run visits the samples in the reference DataLoader's order and
        # Python's `random` stream is left to TrainGridAug's draws
        torch.empty((), dtype=torch.int64).random_()
        idx = list(range(len(self.ds)))
        if self.shuffle:
            seed = int(torch.empty((), dtype=torch.int64).random_().item())
            g = torch.Generator()
            g.manual_seed(seed)
            idx = torch.randperm(len(idx), generator=g).tolist()
        for k in range(len(self)):
            sel = idx[k * self.bs:(k + 1) * self.bs]
            t = torch.as_tensor(sel, device=self.ds.images.device)
            x = self.ds.images.index_select(0, t)
            y = self.ds.labels.index_select(0, t)
            tr = self.ds.transform
            if isinstance(tr, TrainGridAug):
                x, y = tr.batch(x, y, [self.ds.grid_sizes[i] for i in sel])
            yield x.unsqueeze(1), y


class MultiDicomDataModule3D:
    """datasets.py:280-338: volumes from the dataset configs (device-side resize +
    ROI rasterisation), per-sample grid sizes, the class-covering split, train /
    val augmenters and loaders."""

    def __init__(self, configs, batch_size=2, num_frames=5, test_configs=None, frames_reader=None):
        self.configs = configs
        self.test_configs = test_configs
        self.batch_size = batch_size
        self.num_frames = num_frames
        self.frames_reader = frames_reader

    def prepare_data(self):
        pass

    def setup(self, stage=None):
        from .helpers import create_image_and_labels_for_dataset, generate_cumulative_grid_sizes
        xs, ys = [], []
        for cfg in self.configs:
            im, lb = create_image_and_labels_for_dataset(cfg, self.num_frames,
                                                         frames_reader=self.frames_reader)
            xs.append(im)
            ys.append(lb)
        X, Y = torch.cat(xs), torch.cat(ys)
        G = generate_cumulative_grid_sizes(len(X), 10, 0.3)
        tr, va, _te = self.ensure_all_classes_in_training(X, Y, G, NUM_CLASSES)
        aug_train = TrainGridAug(gs_choices=(2, 3, 4, 5), p_grid=1.0, stamp_top_left=True)
        aug_val = TrainGridAug(gs_choices=(2, 3, 4, 5), p_grid=0.0, flip_p=0.0, rot90_p=0.0,
                               jitter_p=0.0, noise_p=0.0, stamp_top_left=False)
        self.train_set = DicomDataset3D(*tr, transform=aug_train)
        self.val_set = DicomDataset3D(*va, transform=aug_val)
        if self.test_configs:
            ims, lbs = zip(*(create_image_and_labels_for_dataset(c, self.num_frames,
                                                                 frames_reader=self.frames_reader)
                             for c in self.test_configs))
            Xt = torch.cat(ims)
            self.test_set = DicomDataset3D(Xt, torch.cat(lbs),
                                           generate_cumulative_grid_sizes(len(Xt), 10, 0.3))

    def train_dataloader(self):
        return DeviceBatchLoader(self.train_set, self.batch_size, shuffle=True)

    def val_dataloader(self):
        return DeviceBatchLoader(self.val_set, self.batch_size, shuffle=False)

    def test_dataloader(self):
        if getattr(self, "test_set", None) is None:
            raise AttributeError("Test dataset not set. Did setup('test') run?")
        return DeviceBatchLoader(self.test_set, self.batch_size, shuffle=False)

    @staticmethod
    def ensure_all_classes_in_training(X, Y, G, num_classes, test_size=0.2, val_size=1.0,
                                       random_state=42):
        """datasets.py:341-364 (same index selection)."""
        n = len(X)
        present = [set(torch.unique(Y[i]).tolist()) for i in range(n)]
        required = set()
        for cls in range(num_classes):
            inds = [i for i in range(n) if cls in present[i]]
            if inds:
                required.add(inds[0])
        remaining = list(set(range(n)) - required)
        np.random.seed(random_state)
        np.random.shuffle(remaining)
        n_train = int(n * (1 - test_size))
        extra = n_train - len(required)
        tr = list(required) + remaining[:extra]
        tv = remaining[extra:]
        nv = int(len(tv) * val_size)
        va, te = tv[:nv], tv[nv:]
        Gt = np.array(G)
        pick = lambda ii: (X[ii], Y[ii], Gt[ii].tolist())  # noqa: E731
        return pick(tr), pick(va), pick(te)
