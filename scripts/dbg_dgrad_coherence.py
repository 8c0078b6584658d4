#!/usr/bin/env python3
"""Debug: does the split-bf16 conv input gradient carry errors that are coherent
over a (d, c) slab?  dy = common-mode C[d, co] + random part; dx for f32 and
bf16x6 vs an fp64 reference: elementwise rms error, bias, and the relative L2
error of the per-(d, ci) sums over (h, w)."""
import math
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spff-unet-spcct_amd")]
from innovative3D import _engine as E  # noqa: E402

DEV = "cuda"


def cl(t):
    return t.permute(0, 2, 3, 4, 1).contiguous()


def run(B, D, H, W, cin, cout, cm, seed=3, scale=1e-9):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(cout, cin, 3, 3, 3, generator=g) / math.sqrt(cin * 27)
    dy = (torch.randn(B, cout, D, H, W, generator=g) + cm * torch.randn(1, cout, D, 1, 1, generator=g)) * scale
    dx64 = torch.nn.grad.conv3d_input((B, cin, D, H, W), w.double(), dy.double(), padding=1)
    L, p, st = E.lib(), E._ptr, E._stream(torch.device(DEV))
    ws = torch.empty(L.spff_conv3d_ws_bytes(B, D, H, W, cin, cout, 3), dtype=torch.uint8, device=DEV)
    dyg, wd = cl(dy).to(DEV), w.to(DEV)
    ref = cl(dx64)
    s64 = ref.sum(dim=(2, 3))
    r = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    sr64 = (ref * r).sum()
    out = []
    for name, m in E.MATH_NAMES.items():
        if name == "bf16x3":
            continue
        dxg = torch.empty(B, D, H, W, cin, device=DEV)
        E.check(L.spff_conv3d_dgrad_ex(p(dyg), p(wd), p(dxg), B, D, H, W, cin, cout, 3, m, p(ws), st), "d")
        torch.cuda.synchronize()
        got = dxg.cpu().double()
        e = got - ref
        s = got.sum(dim=(2, 3))
        out.append(f"{name}: rms {float(e.pow(2).mean().sqrt() / ref.pow(2).mean().sqrt()):.2e} "
                   f"bias {float((e * ref.sign()).mean() / ref.abs().mean()):+.2e} "
                   f"sum_hw relL2 {float((s - s64).norm() / s64.norm()):.2e} "
                   f"sum_hw(e)/sum_hw|ref| {float((s - s64).abs().mean() / ref.abs().sum(dim=(2, 3)).mean()):.2e}")
    print(f"[{B},{D},{H},{W}] {cin}<-{cout} common-mode x{cm}: " + " | ".join(out), flush=True)


for cm in (0.0, 3.0, 30.0):
    run(1, 16, 128, 128, 32, 32, cm)
    run(1, 16, 64, 64, 64, 64, cm)
