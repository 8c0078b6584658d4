#!/usr/bin/env python3
"""Debug: compare the engine's saved per-(b,c) IN affine (al, de) with an fp64
instance norm of its saved conv outputs, for one golden fixture."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "spff-unet-spcct_amd")]
from test_gpu_parity import load, load_core  # noqa: E402
from _golden import state_of  # noqa: E402

d = load(sys.argv[1] if len(sys.argv) > 1 else "fx1_registry_k13")
core = load_core(d)
core.math = "f32"
x = torch.from_numpy(d["x"]).cuda()
lg = core(x)
torch.cuda.synchronize()
plan = core._plan
st = state_of(d)
B, Dd = d["x"].shape[0], d["x"].shape[2]
for blk, lvl in (("enc1", 0), ("bott", 3)):
    for key, j, tag in (("y1", "1", "pre"), ("y2", "2", "body")):
        y = plan.saved(f"{blk}.{key}").double().cpu()
        C = y.shape[1]
        H, W = d["x"].shape[3] >> lvl, d["x"].shape[4] >> lvl
        y = y.view(B, Dd, H, W, C).permute(0, 4, 1, 2, 3)
        al_t = plan.saved(f"{blk}.al{j}")
        print(blk, key, "al raw shape", tuple(al_t.shape))
        al = al_t.double().cpu().reshape(B, C, 1, 1, 1)
        de = plan.saved(f"{blk}.de{j}").double().cpu().reshape(B, C, 1, 1, 1)
        g = torch.from_numpy(st[f"{blk}.{tag}.1.weight"]).double()
        bb = torch.from_numpy(st[f"{blk}.{tag}.1.bias"]).double()
        r64 = F.instance_norm(y, weight=g, bias=bb, eps=1e-5)
        mu = y.mean(dim=(2, 3, 4), keepdim=True)
        var = y.var(dim=(2, 3, 4), unbiased=False, keepdim=True)
        al64 = g.view(1, C, 1, 1, 1) / torch.sqrt(var + 1e-5)
        de64 = bb.view(1, C, 1, 1, 1) - mu * al64
        print(f"  max|al-al64| {float((al - al64).abs().max()):.3e} (|al64| {float(al64.abs().max()):.3e})"
              f"  max|de-de64| {float((de - de64).abs().max()):.3e}")
        print("  al[:4]", al.flatten()[:4].tolist(), "al64[:4]", al64.flatten()[:4].tolist())
        m1 = (y * al + de) > 0
        m2 = r64 > 0
        print(f"  sign disagreements: {int((m1 != m2).sum())} of {m1.numel()}")
