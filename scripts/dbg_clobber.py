#!/usr/bin/env python3
"""Debug: which saved per-(b,c) / per-voxel engine buffers change across a
backward (they should not: the backward only reads them)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "spff-unet-spcct_amd")]
from test_gpu_parity import load, load_core  # noqa: E402
import innovative3D.helpers as Hh  # noqa: E402

d = load(sys.argv[1] if len(sys.argv) > 1 else "fx1_registry_k13")
core = load_core(d)
core.math = "f32"
x = torch.from_numpy(d["x"]).cuda()
y = torch.from_numpy(d["labels"]).cuda()
lg = core(x)
torch.cuda.synchronize()
plan = core._plan
names = [f"{b}.{k}" for b in ("enc1", "enc2", "enc3", "bott", "dec3", "dec2", "dec1")
         for k in ("y1", "a1", "y2", "out", "al1", "de1", "al2", "de2")]
before = {n: plan.saved(n) for n in names}
loss, _ = Hh.ce_dice_with_confusion(lg, y, d["meta"]["K"], 255)
loss.backward()
torch.cuda.synchronize()
for n in names:
    a = plan.saved(n)
    diff = int((a != before[n]).sum())
    if diff:
        print(f"CHANGED {n}: {diff} of {a.numel()} entries")
print("done")
