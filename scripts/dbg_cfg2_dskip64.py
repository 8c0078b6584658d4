#!/usr/bin/env python3
"""Debug: config-2 (or the given shape) engine gradients at the encoder outputs
(grad.dskip0..2) for f32 and bf16x6 math vs the fp64 oracle run with each
engine's own LeakyReLU signs / pool argmaxes.  Per level: max / rms error
relative to max|g|, mean signed error, and the relative L2 error of the
per-(b,c,d) sums over (h,w) (what the FourierGate / SE gradients consume)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spff-unet-spcct_amd"), os.path.join(ROOT, "tests")]
import innovative3D.models as M  # noqa: E402
import innovative3D.helpers as Hh  # noqa: E402
from innovative3D.weightgen import synth_state  # noqa: E402
from innovative3D.synthetic import synthetic_batch  # noqa: E402
from oracle import spff_oracle as O  # noqa: E402
from _kink import forced_branches  # noqa: E402
from test_gpu_parity import engine_branch_masks  # noqa: E402

shape = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "2x5x128x128x128").split("x"))
B, _, D, H, W = shape
torch.set_num_threads(16)
x, y = synthetic_batch(*shape, 13, ignore_frac=0.01, seed=0)
cfg = O.SpffCfg(in_ch=5, num_classes=13, base=32)
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
    eng = {l: core._plan.saved(f"grad.dskip{l}").double().cpu() for l in range(3)}
    egr = {k: p.grad.double().cpu() for k, p in core.named_parameters()}
    masks = engine_branch_masks(core, shape, st, cfg)
    del core
    posts = []
    opost = O._post

    def hpost(P_, xx, stage, cfg_):
        o = opost(P_, xx, stage, cfg_)
        o.retain_grad()
        posts.append(o)
        return o
    O._post = hpost
    try:
        P = O.params_from_state({k: v for k, v in st.items() if not k.endswith("._mask")},
                                dtype=torch.float64)
        with forced_branches(masks):
            O.fwd_bwd(P, x.double(), y, cfg)
    finally:
        O._post = opost
    for l in range(3):
        ref = posts[l].grad.permute(0, 2, 3, 4, 1)  # [B, D, H, W, C]
        C = ref.shape[-1]
        g = eng[l].view(B, D, H >> l, W >> l, C)
        e = g - ref
        sc = float(ref.abs().max())
        sa, sb = ref.sum(dim=(2, 3)), g.sum(dim=(2, 3))
        print(f"{mth:7s} dskip{l}: max {float(e.abs().max()) / sc:.2e} rms {float(e.pow(2).mean().sqrt()) / sc:.2e} "
              f"bias {float((e * ref.sign()).mean()) / float(ref.abs().mean()):+.2e} "
              f"sum_hw relL2 {float((sb - sa).norm() / sa.norm()):.2e}", flush=True)
    rows = []
    for k, pp in P.items():
        kk = k if k in egr else k.replace("freq_mask", "_mask")
        if kk not in egr:
            continue
        r = pp.grad.reshape(-1)
        rows.append((float((egr[kk].reshape(-1) - r).norm() / r.norm().clamp_min(1e-300)), k))
    rows.sort(reverse=True)
    print(f"{mth:7s} grads vs fp64:", " ".join(f"{k}={r:.1e}" for r, k in rows[:6]), flush=True)
