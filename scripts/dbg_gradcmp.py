#!/usr/bin/env python3
"""Debug: dump the engine's parameter gradients (and logits) for one golden
fixture to gpurun_out/grads_<tag>.npz, so runs with different libraries
(SPFF_LIB) or repeated runs can be compared on the host."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "spff-unet-spcct_amd")]
from test_gpu_parity import load, load_core  # noqa: E402
import innovative3D.helpers as Hh  # noqa: E402

name, mth, tag = sys.argv[1], sys.argv[2], sys.argv[3]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
d = load(name)
out = {}
for r in range(reps):
    core = load_core(d)
    core.math = mth
    x = torch.from_numpy(d["x"]).cuda()
    y = torch.from_numpy(d["labels"]).cuda()
    lg = core(x)
    loss, _ = Hh.ce_dice_with_confusion(lg, y, d["meta"]["K"], 255)
    loss.backward()
    torch.cuda.synchronize()
    out[f"r{r}.logits"] = lg.detach().cpu().numpy()
    for k, p in core.named_parameters():
        out[f"r{r}.{k}"] = p.grad.detach().cpu().numpy()
for r in range(1, reps):
    rows = []
    for k in out:
        if k.startswith("r0."):
            a, b = out[k], out["r%d." % r + k[3:]]
            rows.append((float(np.abs(a - b).max() / max(np.abs(a).max(), 1e-30)), k[3:]))
    rows.sort(reverse=True)
    print(f"{tag}: rep {r} vs rep 0, worst rel diffs:", rows[:4])
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed(f"gpurun_out/grads_{tag}.npz", **{k: v for k, v in out.items() if k.startswith("r0.")})
print("saved", tag, len(out))
