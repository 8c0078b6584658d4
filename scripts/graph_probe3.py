#!/usr/bin/env python3
"""Diagnostics: where a HIP-graph replay of the SPFF training step departs from the eager
step (runner.step only -- no autograd graph kept alive across steps)."""
import pathlib
import sys

import torch

MATH = sys.argv[1] if len(sys.argv) > 1 else "f16x3"

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "spff-unet-spcct_amd")]
import innovative3D.models as M  # noqa: E402
from innovative3D.distributed import DataParallelSPFF  # noqa: E402
from innovative3D.synthetic import synthetic_batch  # noqa: E402
from innovative3D.weightgen import synth_state  # noqa: E402

K, D = 13, 16
core = M.build_spct_energyfilm_fourier(num_classes=K, base=16, in_channels=5)
for b in core._blocks():
    b.fgate._ensure_mask(D, "cpu")
st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=11)
core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
core = core.to("cuda")
core.math = MATH
runner = DataParallelSPFF(core, K, 255)
x1, y1 = synthetic_batch(2, 5, D, 32, 48, num_classes=K, ignore_frac=0.02, seed=1)
x2, y2 = synthetic_batch(2, 5, D, 32, 48, num_classes=K, ignore_frac=0.02, seed=2)
x, y = x1.cuda(), y1.cuda()


def snap(loss, conf):
    torch.cuda.synchronize()
    return (float(loss), conf.clone(), runner.last_logits.clone(),
            {k: p.grad.clone() for k, p in core.named_parameters()})


refs = {}
for tag, (xx, yy) in (("x1", (x1, y1)), ("x2", (x2, y2))):
    x.copy_(xx)
    y.copy_(yy)
    l, c = runner.step(x, y)
    refs[tag] = snap(l, c)
    print(f"eager {tag}: loss {refs[tag][0]:.7f}", flush=True)
x.copy_(x1)
y.copy_(y1)
for _ in range(2):
    runner.step(x, y)
torch.cuda.synchronize()
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    runner.step(x, y)
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    gl, gc = runner.step(x, y)
glg = runner.last_logits
print("captured", MATH, flush=True)
plan = core._plan
ws = plan._ws


def ranges(a, b):
    """coalesced differing 4-byte word ranges of two byte tensors"""
    d = (a.view(torch.int32) != b.view(torch.int32)).nonzero().flatten().cpu().tolist()
    out = []
    for i in d:
        if out and i <= out[-1][1] + 64:
            out[-1][1] = i
        else:
            out.append([i, i])
    return [(4 * lo, 4 * (hi - lo + 1)) for lo, hi in out]


x.copy_(x1)
y.copy_(y1)
runner.step(x, y)
torch.cuda.synchronize()
ws_e = ws.clone()
flat_e = core._flat.clone()
for tag, (xx, yy) in (("x1", (x1, y1)), ("x1", (x1, y1)), ("x2", (x2, y2)), ("x1", (x1, y1))):
    x.copy_(xx)
    y.copy_(yy)
    g.replay()
    torch.cuda.synchronize()
    r = refs[tag]
    if tag == "x1":
        rg = ranges(ws, ws_e)
        print(f"  ws diff vs eager x1: {len(rg)} ranges {rg[:12]} flat equal "
              f"{torch.equal(core._flat, flat_e)}", flush=True)
    dl = float((glg - r[2]).abs().max())
    dg = max(float((p.grad - r[3][k]).abs().max()) for k, p in core.named_parameters())
    print(f"replay {tag}: loss {float(gl):.7f} (eager {r[0]:.7f}) |dlogit| {dl:.3e} conf "
          f"{torch.equal(gc, r[1])} max|dgrad| {dg:.3e}", flush=True)
x.copy_(x1)
y.copy_(y1)
l, c = runner.step(x, y)
torch.cuda.synchronize()
print(f"eager after replays x1: loss {float(l):.7f} logits equal "
      f"{torch.equal(runner.last_logits, refs['x1'][2])} ws ranges {ranges(ws, ws_e)[:12]}",
      flush=True)
print("ws bytes", ws.numel(), flush=True)
