"""The data-path oracle (oracle/data_oracle.py) against fixtures produced by the
reference's own functions (tests/golden/make_golden_data.py): stripe shuffle,
TrainGridAug (noise off), ellipse-ROI rasterisation, cumulative grid sizes."""
import json
import pathlib
import random

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import data_oracle as DO

FX = np.load(pathlib.Path(__file__).parent / "golden" / "data_aug.npz")
META = json.loads(bytes(FX["meta"]).decode())


@pytest.mark.parametrize("k", range(4))
def test_shuffle_stripes_matches_reference(k):
    H, W, gr, gc, seed = META["stripes"][k]
    x, y = torch.from_numpy(FX[f"st{k}_x"]), torch.from_numpy(FX[f"st{k}_y"])
    xo, yo = DO.shuffle_stripes(x, y, gr, gc, random.Random(seed))
    assert np.array_equal(xo.numpy(), FX[f"st{k}_xo"])
    assert np.array_equal(yo.numpy(), FX[f"st{k}_yo"])


@pytest.mark.parametrize("k", range(6))
def test_train_grid_aug_matches_reference(k):
    H, W, gs, seed, flip_p, rot_p, jit_p = META["aug"][k]
    x, y = torch.from_numpy(FX[f"aug{k}_x"]), torch.from_numpy(FX[f"aug{k}_y"])
    d = DO.draw_aug(random.Random(seed), H, W, None if gs < 0 else gs, flip_p=flip_p,
                    rot90_p=rot_p, jitter_p=jit_p, noise_p=0.0)
    xo, yo = DO.train_grid_aug(x.clone(), y.clone(), d)
    assert np.array_equal(xo.numpy(), FX[f"aug{k}_xo"])
    assert np.array_equal(yo.numpy(), FX[f"aug{k}_yo"])


@pytest.mark.parametrize("k", range(2))
def test_rasterize_matches_reference(k):
    F_, H, W = META["rois"][k]
    rois = [tuple(int(v) for v in r) for r in FX[f"roi{k}_rois"]]
    assert np.array_equal(DO.rasterize_rois(rois, F_, H, W).numpy(), FX[f"roi{k}_labels"])


@pytest.mark.parametrize("k", range(2))
def test_cumulative_grid_sizes_matches_reference(k):
    n, g, p, seed = META["grids"][k]
    assert DO.cumulative_grid_sizes(n, g, p, random.Random(seed)) == FX[f"grid{k}"].tolist()


def test_rot90_convention():
    """The device gather's inverse map of torch.rot90(x, k, dims=(-2,-1))."""
    x = torch.arange(3 * 5).view(3, 5)
    H, W = x.shape
    for k in (1, 2, 3):
        r = torch.rot90(x, k, dims=(0, 1))
        for i in range(r.shape[0]):
            for j in range(r.shape[1]):
                if k == 1:
                    src = (j, W - 1 - i)
                elif k == 2:
                    src = (H - 1 - i, W - 1 - j)
                else:
                    src = (H - 1 - j, i)
                assert r[i, j] == x[src]


def test_resize_is_interpolate_antialias():
    t = torch.rand(2, 13, 26)
    ref = F.interpolate(t.unsqueeze(1), size=(5, 7), mode="bilinear", align_corners=False,
                        antialias=True).squeeze(1)
    assert torch.equal(DO.resize_frames(t, 5, 7), ref)


def test_device_batch_loader_order_matches_torch_dataloader():
    """DeviceBatchLoader(shuffle=True) visits samples in the order the reference's
    DataLoader(shuffle=True) draws (datasets.py:318-323: RandomSampler on torch's
    default generator) for the same torch seed."""
    import torch
    from innovative3D.datasets import DeviceBatchLoader
    n = 11

    class _DS:
        images = torch.arange(n, dtype=torch.float32).view(n, 1, 1, 1)
        labels = torch.zeros(n, 1, 1, 1, dtype=torch.int64)
        transform = None

        def __len__(self):
            return n

        def __getitem__(self, i):
            return i
    for seed in (0, 7):
        torch.manual_seed(seed)
        ref = [int(i) for b in torch.utils.data.DataLoader(_DS(), batch_size=3, shuffle=True)
               for i in b]
        after_ref = torch.rand(1)
        torch.manual_seed(seed)
        got = [int(v) for x, _y in DeviceBatchLoader(_DS(), 3, True) for v in x.reshape(-1)]
        assert got == ref
        assert torch.equal(torch.rand(1), after_ref)  # same number of default-generator draws
