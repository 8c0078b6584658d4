#!/usr/bin/env python3
"""Diagnostics: HIP-graph capture of the training step vs eager (tests/test_gpu_graph.py)."""
import pathlib
import sys

import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "spff-unet-spcct_amd")]
import innovative3D.models as M  # noqa: E402
import innovative3D.helpers as Hh  # noqa: E402
from innovative3D.synthetic import synthetic_batch  # noqa: E402
from innovative3D.weightgen import synth_state  # noqa: E402

mth = sys.argv[1] if len(sys.argv) > 1 else "f16x3"
second = len(sys.argv) > 2 and sys.argv[2] == "2"
K, D = 13, 16
core = M.build_spct_energyfilm_fourier(num_classes=K, base=16, in_channels=5)
for b in core._blocks():
    b.fgate._ensure_mask(D, "cpu")
st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=11)
core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
core = core.to("cuda")
core.math = mth
x1, y1 = synthetic_batch(2, 5, D, 32, 48, num_classes=K, ignore_frac=0.02, seed=1)
x2, y2 = synthetic_batch(2, 5, D, 32, 48, num_classes=K, ignore_frac=0.02, seed=2)
x, y = x1.cuda(), y1.cuda()


def step():
    for p in core.parameters():
        p.grad = None
    lg = core(x)
    loss, conf, ce = Hh.ce_dice_parts(lg, y, K, 255)
    loss.backward()
    return lg, loss, conf, ce


lg, loss, conf, ce = step()
torch.cuda.synchronize()
ref = (lg.detach().clone(), float(loss), conf.clone(), float(ce),
       {k: p.grad.clone() for k, p in core.named_parameters()})
print(f"eager x1: loss {ref[1]:.7f} ce {ref[3]:.7f}")
if second:
    x.copy_(x2)
    y.copy_(y2)
    _lg, l2, _c, ce2 = step()
    torch.cuda.synchronize()
    print(f"eager x2: loss {float(l2):.7f} ce {float(ce2):.7f}")
    x.copy_(x1)
    y.copy_(y1)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    step()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    glg, gloss, gconf, gce = step()
for r in range(3):
    g.replay()
    torch.cuda.synchronize()
    dlg = float((glg - ref[0]).abs().max())
    gr = {k: p.grad for k, p in core.named_parameters()}
    dg = max(float((gr[k] - ref[4][k]).abs().max()) for k in gr)
    print(f"replay {r}: loss {float(gloss):.7f} ce {float(gce):.7f} |dlogit| {dlg:.3e} "
          f"conf equal {torch.equal(gconf, ref[2])} max|dgrad| {dg:.3e}")
