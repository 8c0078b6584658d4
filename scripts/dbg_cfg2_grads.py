#!/usr/bin/env python3
"""Debug: one config-2 engine step (2 x 5 x 128^3, K 13, base 32, weightgen seed 0,
synthetic_batch seed 0) under --math; dumps every parameter gradient to
gpurun_out/cfg2_<tag>.npz.  Runs with SPFF_DEBUG_SPLIT set to subsets of
fwd,dgrad,wgrad localise a precision difference between the arithmetics."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spff-unet-spcct_amd")]
import innovative3D.models as M  # noqa: E402
import innovative3D.helpers as Hh  # noqa: E402
from innovative3D.weightgen import synth_state  # noqa: E402
from innovative3D.synthetic import synthetic_batch  # noqa: E402

mth, tag = sys.argv[1], sys.argv[2]
shape = tuple(int(v) for v in (sys.argv[3].split("x") if len(sys.argv) > 3 else "2x5x128x128x128".split("x")))
core = M.build_spct_energyfilm_fourier(num_classes=13, base=32, in_channels=5)
for b in core._blocks():
    b.fgate._ensure_mask(shape[2], "cpu")
st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=0)
core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
core = core.cuda()
core.math = mth
x, y = synthetic_batch(*shape, 13, ignore_frac=0.01, seed=0)
lg = core(x.cuda())
loss, _ = Hh.ce_dice_with_confusion(lg, y.cuda(), 13, 255)
loss.backward()
torch.cuda.synchronize()
os.makedirs("gpurun_out", exist_ok=True)
np.savez(f"gpurun_out/cfg2_{tag}.npz", **{k: p.grad.detach().cpu().numpy()
                                          for k, p in core.named_parameters()})
print(tag, "loss", float(loss), "split dirs", os.environ.get("SPFF_DEBUG_SPLIT", "all"))
