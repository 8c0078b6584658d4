"""Device data path (csrc/data.hip, innovative3D/datasets.py) against the
fixtures the reference's own functions produced (tests/golden/data_aug.npz) and
the oracle: bit-exact stripe shuffle, TrainGridAug (noise off) and ROI
rasterisation; the antialiased resize within 2e-6 of F.interpolate; the noise
branch statistically (its values come from a device RNG, not torch.randn_like)."""
import json
import pathlib
import random

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import innovative3D.datasets as DS
from innovative3D import _engine as E
from oracle import data_oracle as DO

pytestmark = pytest.mark.gpu
DEV = "cuda"
FX = np.load(pathlib.Path(__file__).parent / "golden" / "data_aug.npz")
META = json.loads(bytes(FX["meta"]).decode())


@pytest.mark.parametrize("k", range(4))
def test_device_stripe_shuffle(k):
    H, W, gr, gc, seed = META["stripes"][k]
    x = torch.from_numpy(FX[f"st{k}_x"]).to(DEV)
    y = torch.from_numpy(FX[f"st{k}_y"]).to(DEV)
    random.seed(seed)
    xo, yo = DS._shuffle_stripes(x, y, gr, gc)
    assert np.array_equal(xo.cpu().numpy(), FX[f"st{k}_xo"])
    assert np.array_equal(yo.cpu().numpy(), FX[f"st{k}_yo"])


@pytest.mark.parametrize("k", range(6))
def test_device_train_grid_aug(k):
    H, W, gs, seed, flip_p, rot_p, jit_p = META["aug"][k]
    x = torch.from_numpy(FX[f"aug{k}_x"]).to(DEV)
    y = torch.from_numpy(FX[f"aug{k}_y"]).to(DEV)
    aug = DS.TrainGridAug(gs_choices=(2, 3, 4, 5), p_grid=1.0, flip_p=flip_p, rot90_p=rot_p,
                          jitter_p=jit_p, noise_p=0.0, stamp_top_left=True)
    random.seed(seed)
    xo, yo = aug(x, y, None if gs < 0 else gs)
    torch.cuda.synchronize()
    assert np.array_equal(xo.cpu().numpy(), FX[f"aug{k}_xo"])
    assert np.array_equal(yo.cpu().numpy(), FX[f"aug{k}_yo"])


def test_device_aug_batch_matches_oracle_and_noise_stats():
    torch.manual_seed(0)
    B, F_, H, W = 6, 5, 64, 64
    x = 2 * torch.randn(B, F_, H, W)
    y = torch.randint(0, 13, (B, F_, H, W))
    aug = DS.TrainGridAug(noise_p=0.0)
    random.seed(21)
    xo, yo = aug.batch(x.to(DEV), y.to(DEV), [None, 2, 3, 1, 5, 4])
    rng = random.Random(21)
    for b, gs in enumerate([None, 2, 3, 1, 5, 4]):
        d = DO.draw_aug(rng, H, W, gs, noise_p=0.0)
        rx, ry = DO.train_grid_aug(x[b:b + 1].clone(), y[b].clone(), d)
        assert torch.equal(xo[b].cpu(), rx[0]) and torch.equal(yo[b].cpu(), ry)
    # noise on: same decisions plus N(0, min(0.01, 0.25 std)) per voxel
    aug_n = DS.TrainGridAug(noise_p=1.0, p_grid=0.0, flip_p=0.0, rot90_p=0.0, jitter_p=0.0,
                            stamp_top_left=False)
    xb = x.to(DEV)
    random.seed(3)
    xn, _ = aug_n.batch(xb, None, [1] * B)
    d = (xn - xb).cpu()
    exp = min(0.01, 0.25 * float(x[0].std()))
    assert abs(float(d[0].std()) / exp - 1) < 0.02 and abs(float(d[0].mean())) < 5e-4


@pytest.mark.parametrize("k", range(2))
def test_device_rasterize(k):
    F_, H, W = META["rois"][k]
    rois = torch.from_numpy(FX[f"roi{k}_rois"]).to(DEV)
    lab = E.rasterize_ellipses(rois, F_, H, W)
    assert np.array_equal(lab.cpu().numpy(), FX[f"roi{k}_labels"])


@pytest.mark.parametrize("shape", [(3, 1300, 1300, 512, 512), (2, 97, 131, 40, 50),
                                   (2, 20, 30, 45, 70)])
def test_device_resize_antialias(shape):
    n, h, w, H, W = shape
    g = torch.Generator().manual_seed(1)
    t = torch.rand(n, h, w, generator=g) * 1000
    ref = DO.resize_frames(t, H, W)
    out = E.resize_bilinear_aa(t.to(DEV), H, W).cpu()
    assert float((out - ref).abs().max()) <= 2e-6 * float(ref.abs().max())
