#!/usr/bin/env python3
"""Generate the data-path golden fixtures by running the REFERENCE's own
functions (container-only; the reference never travels to the GPU box):

    python tests/golden/make_golden_data.py      # writes tests/golden/data_aug.npz

Uses make_golden.py's harness (stub modules for the absent pytorch_lightning /
torchvision / pydicom, /root/reference on sys.path) and calls, with the
module-level ``random`` seeded per case:
* innovative3D.datasets._shuffle_stripes (datasets.py:60-115);
* innovative3D.datasets.TrainGridAug.__call__ (datasets.py:158-209) with the
  noise off (torch.randn_like draws cannot be reproduced by a device RNG);
* innovative3D.helpers.is_pixel_in_ellipse over ROI boxes, in the loop order of
  create_image_and_labels_for_dataset (helpers.py:199-204), whose DICOM read
  itself needs pydicom;
* innovative3D.helpers.generate_cumulative_grid_sizes (helpers.py:280-289).
Every fixture stores inputs and outputs."""
from __future__ import annotations

import json
import pathlib
import random
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
import make_golden as MG  # noqa: E402


def main():
    MG._install_harness()
    import torch
    import innovative3D.datasets as D  # noqa: E402  (the reference's)
    import innovative3D.helpers as Hh  # noqa: E402
    assert pathlib.Path(D.__file__).resolve().is_relative_to(MG.REF.resolve()), D.__file__
    out = {}
    meta = {"stripes": [], "aug": [], "rois": [], "grids": []}
    rng = np.random.default_rng(7)
    # stripe shuffles, ragged sizes
    for k, (H, W, gr, gc, seed) in enumerate([(13, 17, 3, 5, 1), (20, 24, 4, 4, 2),
                                              (11, 9, 2, 1, 3), (16, 16, 5, 5, 4)]):
        x = torch.from_numpy(rng.standard_normal((1, 3, H, W)).astype(np.float32))
        y = torch.from_numpy(rng.integers(0, 13, size=(3, H, W)).astype(np.int64))
        random.seed(seed)
        xo, yo = D._shuffle_stripes(x, y, gr, gc)
        out[f"st{k}_x"], out[f"st{k}_y"] = x.numpy(), y.numpy()
        out[f"st{k}_xo"], out[f"st{k}_yo"] = xo.numpy(), yo.numpy()
        meta["stripes"].append([H, W, gr, gc, seed])
    # full TrainGridAug calls (noise off), square and non-square, gs given / drawn
    cases = [(40, 40, 3, 11, 0.5, 0.5, 0.3), (40, 40, None, 12, 0.5, 0.5, 0.3),
             (36, 44, 5, 13, 1.0, 1.0, 1.0), (48, 48, 2, 14, 0.0, 1.0, 1.0),
             (33, 35, 4, 15, 1.0, 0.0, 0.0), (64, 64, 1, 16, 0.5, 0.5, 0.5)]
    for k, (H, W, gs, seed, flip_p, rot_p, jit_p) in enumerate(cases):
        x = torch.from_numpy((3 * rng.standard_normal((1, 5, H, W))).astype(np.float32))
        y = torch.from_numpy(rng.integers(0, 13, size=(5, H, W)).astype(np.int64))
        aug = D.TrainGridAug(gs_choices=(2, 3, 4, 5), p_grid=1.0, flip_p=flip_p, rot90_p=rot_p,
                             jitter_p=jit_p, noise_p=0.0, stamp_top_left=True)
        random.seed(seed)
        xo, yo = aug(x.clone(), y.clone(), gs)
        out[f"aug{k}_x"], out[f"aug{k}_y"] = x.numpy(), y.numpy()
        out[f"aug{k}_xo"], out[f"aug{k}_yo"] = xo.numpy(), yo.numpy()
        meta["aug"].append([H, W, -1 if gs is None else gs, seed, flip_p, rot_p, jit_p])
    # ellipse ROI rasterisation (the loop of create_image_and_labels_for_dataset)
    for k, rois in enumerate([[(3, 4, 11, 7, 2), (8, 2, 9, 13, 5), (20, 20, 1, 1, 3)],
                              [(0, 0, 31, 29, 1), (10, 12, 12, 6, 4), (25, 1, 6, 30, 7)]]):
        F_, H, W = 2, 32, 32
        lb = np.zeros((F_, H, W), dtype=np.int64)
        for f in range(F_):
            for (x0, y0, w0, h0, lab) in rois:
                for px in range(x0, x0 + w0):
                    for py in range(y0, y0 + h0):
                        if Hh.is_pixel_in_ellipse(px, py, (x0, y0, w0, h0)):
                            lb[f, py, px] = lab
        out[f"roi{k}_labels"] = lb
        out[f"roi{k}_rois"] = np.array(rois, dtype=np.int32)
        meta["rois"].append([F_, H, W])
    for k, (n, g, p, seed) in enumerate([(37, 10, 0.3, 5), (25, 4, 0.2, 6)]):
        random.seed(seed)
        out[f"grid{k}"] = np.array(Hh.generate_cumulative_grid_sizes(n, g, p), dtype=np.int64)
        meta["grids"].append([n, g, p, seed])
    out["meta"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(HERE / "data_aug.npz", **out)
    print("wrote", HERE / "data_aug.npz", len(out))


if __name__ == "__main__":
    main()
