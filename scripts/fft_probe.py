#!/usr/bin/env python3
"""Run-to-run check of torch.fft.rfft / irfft in fp64 on the GPU (hipFFT / rocFFT) for the
FourierGate's shapes: the spectrum of s[B, 1, D, 1, 1] along dim 2 and its irfft(n=D),
forward and backward, repeated and compared with the host evaluation.

    python scripts/fft_probe.py [D ...]"""
import sys

import torch

Ds = [int(a) for a in sys.argv[1:]] or [5, 8, 16, 7, 128]
torch.manual_seed(0)
for D in Ds:
    s0 = torch.randn(1, 1, D, 1, 1, dtype=torch.float64)
    M = torch.rand(D // 2 + 1, dtype=torch.float64)
    g = torch.randn(1, 1, D, 1, 1, dtype=torch.float64)

    def run(dev):
        s = s0.detach().to(dev).clone().requires_grad_(True)
        Sf = torch.fft.rfft(s, dim=2)
        w = torch.fft.irfft(Sf * M.to(dev).view(1, 1, -1, 1, 1), n=D, dim=2)
        (w * g.to(dev)).sum().backward()
        return w.detach().cpu(), s.grad.cpu()

    w_h, g_h = run("cpu")
    worst_w = worst_g = 0.0
    for _ in range(50):
        w_d, g_d = run("cuda")
        worst_w = max(worst_w, float((w_d - w_h).abs().max() / w_h.abs().max()))
        worst_g = max(worst_g, float((g_d - g_h).abs().max() / g_h.abs().max()))
    print(f"D={D:4d}: 50 device runs vs host: max rel err w {worst_w:.2e}, ds {worst_g:.2e}",
          flush=True)
