#!/usr/bin/env python3
"""Debug: stage-wise comparison of the SwinUNETR engine's saved tensors with the
oracle's (fp64), to localise a mismatch.  Usage: dbg_swin.py [B D H W] [math]"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "spff-unet-spcct_amd")]
from test_gpu_swin import _case, _engine_model  # noqa: E402
from oracle import swin_oracle as S  # noqa: E402

B, D, H, W = (int(a) for a in sys.argv[1:5]) if len(sys.argv) > 4 else (1, 32, 32, 32)
mth = sys.argv[5] if len(sys.argv) > 5 else "f32"
K = 9
cfg, st, x, y = _case(B, D, H, W, K, seed=3)
m = _engine_model(st, K, mth)
lg = m(x.cuda())
torch.cuda.synchronize()
plan = m._plan(x.cuda())
P = S.params_from_state(st, dtype=torch.float64, requires_grad=False)
taps = {}
with torch.no_grad():
    ref = S.forward(P, x.double(), cfg, taps=taps)


def cl(t):  # [B, C, D, H, W] -> [V, C]
    return t.permute(0, 2, 3, 4, 1).reshape(-1, t.shape[1])


def cmp(name, mine, r):
    e = float((mine.double() - r).abs().max())
    print(f"{name:24s} max|d| {e:.3e}   max|ref| {float(r.abs().max()):.3e}", flush=True)


cmp("t0", plan.saved("t0").cpu(), cl(taps["x0"]))
for l in range(5):
    cmp(f"hs{l}", plan.saved(f"hs{l}").cpu(), cl(taps["hs"][l]))
for nm, key in (("encoder1.layer.out", "enc0"), ("encoder2.layer.out", "enc1"),
                ("encoder3.layer.out", "enc2"), ("encoder4.layer.out", "enc3"),
                ("encoder10.layer.out", "dec4"), ("decoder5.conv_block.out", "dec3"),
                ("decoder4.conv_block.out", "dec2"), ("decoder3.conv_block.out", "dec1"),
                ("decoder2.conv_block.out", "dec0"), ("decoder1.conv_block.out", "out")):
    cmp(nm, plan.saved(nm).cpu(), cl(taps[key]))
cmp("logits", lg.detach().cpu(), ref)
