#!/usr/bin/env python3
"""Data-path throughput: the device TrainGridAug (one fused gather + noise +
stamp per batch) and ROI rasterisation / resize, against the CPU restatement of
the reference's per-sample TrainGridAug (oracle/data_oracle.py) on the host.
Prints one JSON line."""
import json
import os
import random
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spff-unet-spcct_amd")]
import innovative3D.datasets as DS  # noqa: E402
from innovative3D import _engine as E  # noqa: E402
from oracle import data_oracle as DO  # noqa: E402

B, F_, H, W = 16, 5, 512, 512
dev = torch.device("cuda")
x = torch.randn(B, F_, H, W, device=dev)
y = torch.randint(0, 13, (B, F_, H, W), device=dev)
aug = DS.TrainGridAug()
random.seed(0)
for _ in range(3):
    aug.batch(x, y, [None] * B)
torch.cuda.synchronize()
n = 20
t0 = time.perf_counter()
for _ in range(n):
    aug.batch(x, y, [None] * B)
torch.cuda.synchronize()
gpu_s = (time.perf_counter() - t0) / n
rois = torch.tensor([(40 + 30 * i, 60 + 25 * i, 80, 70, i % 12 + 1) for i in range(12)],
                    dtype=torch.int32, device=dev)
frames = torch.rand(5, 1300, 1300, device=dev) * 4000
E.rasterize_ellipses(rois, 5, 512, 512)
E.resize_bilinear_aa(frames, 512, 512)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    E.rasterize_ellipses(rois, 5, 512, 512)
    E.resize_bilinear_aa(frames, 512, 512)
torch.cuda.synchronize()
vol_s = (time.perf_counter() - t0) / n
# CPU: the reference's per-sample TrainGridAug (its DataLoader workers run this)
torch.set_num_threads(1)
xc, yc = x[:4].cpu(), y[:4].cpu()
rng = random.Random(0)
t0 = time.perf_counter()
for b in range(4):
    d = DO.draw_aug(rng, H, W, None)
    DO.train_grid_aug(xc[b:b + 1].clone(), yc[b].clone(), d)
cpu_s = (time.perf_counter() - t0) / 4
rl = [tuple(int(v) for v in r) for r in rois.cpu()]
t0 = time.perf_counter()
DO.rasterize_rois(rl, 1, 512, 512)
ras_cpu_s = time.perf_counter() - t0
print(json.dumps({
    "workload": f"TrainGridAug on {B} x {F_} x {H} x {W} (image + labels) per batch",
    "gpu_samples_per_s": B / gpu_s, "gpu_ms_per_batch": gpu_s * 1e3,
    "gpu_GBps": B * F_ * H * W * (4 + 8) * 2 / gpu_s / 1e9,
    "cpu_samples_per_s_1thread": 1 / cpu_s,
    "volume_build_ms_gpu": vol_s * 1e3,
    "volume_build_note": "5 frames 1300^2 -> 512^2 resize + 12-ROI rasterisation",
    "rasterise_one_frame_cpu_python_ms": ras_cpu_s * 1e3,
}), flush=True)
