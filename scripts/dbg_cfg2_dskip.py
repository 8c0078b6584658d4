#!/usr/bin/env python3
"""Debug: config-2 step with f32 and with bf16x6 math in ONE process (run it with
SPFF_DEBUG_SPLIT=dgrad so both forwards are bitwise equal); compares the
engine's gradient at the three encoder outputs (grad.dskip0..2) per depth:
rms and mean signed difference relative to max|g|."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spff-unet-spcct_amd")]
import innovative3D.models as M  # noqa: E402
import innovative3D.helpers as Hh  # noqa: E402
from innovative3D.weightgen import synth_state  # noqa: E402
from innovative3D.synthetic import synthetic_batch  # noqa: E402

shape = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2x5x128x128x128").split("x"))
B, _, D, H, W = shape
x, y = synthetic_batch(*shape, 13, ignore_frac=0.01, seed=0)
res = {}
for mth in ("f32", "bf16x6"):
    core = M.build_spct_energyfilm_fourier(num_classes=13, base=32, in_channels=5)
    for b in core._blocks():
        b.fgate._ensure_mask(D, "cpu")
    st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=0)
    core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    core = core.cuda()
    core.math = mth
    lg = core(x.cuda())
    loss, _ = Hh.ce_dice_with_confusion(lg, y.cuda(), 13, 255)
    loss.backward()
    torch.cuda.synchronize()
    res[mth] = ({l: core._plan.saved(f"grad.dskip{l}").double().cpu() for l in range(3)},
                {k: p.grad.double().cpu() for k, p in core.named_parameters()}, float(loss))
    del core
print("loss", res["f32"][2], res["bf16x6"][2])
for l in range(3):
    a, b = res["f32"][0][l], res["bf16x6"][0][l]
    C = a.shape[1]
    a = a.view(B, D, H >> l, W >> l, C)
    b = b.view(B, D, H >> l, W >> l, C)
    e = b - a
    sc = float(a.abs().max())
    print(f"dskip{l}: max|g| {sc:.3e} max|e| {float(e.abs().max()) / sc:.2e} rms {float(e.pow(2).mean().sqrt()) / sc:.2e}"
          f" bias(e*sign g) {float((e * a.sign()).mean()) / float(a.abs().mean()):+.2e}")
    pd = e.pow(2).mean(dim=(0, 2, 3, 4)).sqrt() / sc
    print("   per-d rms: " + " ".join(f"{float(v):.1e}" for v in pd[:8]) + " ... " +
          " ".join(f"{float(v):.1e}" for v in pd[-4:]))
    pc = e.pow(2).mean(dim=(0, 1, 2, 3)).sqrt() / sc
    print("   per-c rms: " + " ".join(f"{float(v):.1e}" for v in pc[:16]))
    # relative error of the fgate-like cancelling sums sum_hw g (per b, c, d)
    sa = a.sum(dim=(2, 3))
    sb = b.sum(dim=(2, 3))
    print(f"   sum_hw: rel L2 {float((sb - sa).norm() / sa.norm()):.2e}")
rows = []
for k, g in res["f32"][1].items():
    gb = res["bf16x6"][1][k]
    rows.append((float((gb - g).norm() / g.norm().clamp_min(1e-30)), k))
rows.sort(reverse=True)
print("grads:", " ".join(f"{k}={r:.1e}" for r, k in rows[:6]))
