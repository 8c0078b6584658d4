#!/usr/bin/env python3
"""Correctness of PyTorch's fp64 device reductions at the oracle's shapes, with DIFFERENT
data on every call (a reduction that read another call's stale partial sums would still
repeat itself on identical data): x.sum(dim=(1, 3, 4)) (the FourierGate / SpectralSE
pool and its broadcast backward), x.sum(dim=(2, 3, 4)) (the SE pool), x.sum(dim=(3, 4))
(EnergyFiLM) of [1, C, 5, H, W] tensors, each compared with the host result.  Diagnostics.

    python scripts/reduce_det_probe.py [REPS]"""
import sys

import torch

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
torch.manual_seed(0)
for dt in (torch.float64, torch.float32):
    for C, H in ((32, 512), (64, 256), (128, 128), (256, 64)):
        for dims in ((1, 3, 4), (2, 3, 4), (3, 4)):
            nbad, worst = 0, 0.0
            for _ in range(reps):
                xh = torch.randn(1, C, 5, H, H, dtype=dt)
                r = xh.cuda().sum(dim=dims).cpu()
                ref = xh.double().sum(dim=dims)
                err = float((r.double() - ref).abs().max() / ref.abs().max())
                tol = 1e-12 if dt == torch.float64 else 1e-4
                if err > tol:
                    nbad += 1
                    worst = max(worst, err)
            print(f"{str(dt)[6:]} [1,{C},5,{H},{H}] sum{dims}: {nbad}/{reps} wrong "
                  f"(worst {worst:.2e})", flush=True)
