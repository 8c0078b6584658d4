"""Unsharded engine gradients at the depth-sharded test's shape (1 x 5 x 16 x 32 x 32,
base 8, bf16x6) saved to gpurun_out/ab_grads_<tag>.npz -- run once per library
(SPFF_LIB) and compare: python scripts/ab_grads.py <tag> [compare_tag]"""
import pathlib
import sys

import numpy as np
import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "spff-unet-spcct_amd")]
from test_gpu_sharded import _data, _model  # noqa: E402

import innovative3D.helpers as Hh  # noqa: E402

tag = sys.argv[1]
out = ROOT / "gpurun_out"
out.mkdir(exist_ok=True)
if tag != "-":
    core = _model("bf16x6", 16)
    x, y = _data(16)
    logits = core(x.cuda())
    loss, conf = Hh.ce_dice_with_confusion(logits, y.cuda(), 5, 255)
    loss.backward()
    np.savez(out / f"ab_grads_{tag}.npz", logits=logits.detach().cpu().numpy(),
             **{"g_" + k: p.grad.cpu().numpy() for k, p in core.named_parameters() if p.grad is not None})
if len(sys.argv) > 2:
    a, b = np.load(out / f"ab_grads_{sys.argv[2]}.npz"), np.load(out / f"ab_grads_{sys.argv[3]}.npz")
    print("logits", float(np.abs(a["logits"] - b["logits"]).max()))
    rows = sorted(((float(np.abs(a[k] - b[k]).max()) / max(float(np.abs(b[k]).max()), 1e-30), k)
                   for k in a.files if k.startswith("g_")), reverse=True)
    print(rows[:6])
