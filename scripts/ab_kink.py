"""Engine gradients at the depth-sharded test's shape (1 x 5 x 16 x 32 x 32, base 8,
bf16x6) against the fp64 oracle run with the ENGINE's own LeakyReLU signs and pool
argmaxes (tests/_kink.forced_branches): the branch-consistent check for a library
variant (SPFF_LIB).  Prints the worst gradient error relative to max|g64|."""
import pathlib
import sys

import torch

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests"), str(ROOT / "spff-unet-spcct_amd")]
from test_gpu_sharded import _data, _model  # noqa: E402
from test_gpu_parity import engine_branch_masks  # noqa: E402
from _kink import forced_branches  # noqa: E402
from oracle import spff_oracle as O  # noqa: E402

import innovative3D.helpers as Hh  # noqa: E402

core = _model("bf16x6", 16)
x, y = _data(16)
logits = core(x.cuda())
loss, _conf = Hh.ce_dice_with_confusion(logits, y.cuda(), 5, 255)
loss.backward()
torch.cuda.synchronize()
st = {k: v.detach().cpu().numpy() for k, v in core.state_dict().items()}
cfg = O.SpffCfg(in_ch=5, num_classes=5, base=8)
masks = engine_branch_masks(core, tuple(x.shape), st, cfg)
P = O.params_from_state({k: v for k, v in st.items() if not k.endswith("._mask")},
                        dtype=torch.float64)
with forced_branches(masks):
    O.fwd_bwd(P, x.double(), y, cfg)
grads = dict(core.named_parameters())
rows = []
for k, v in P.items():
    if v.grad is None or k not in grads or grads[k].grad is None:
        continue
    g64 = v.grad.reshape(-1)
    g = grads[k].grad.detach().double().cpu().reshape(-1)
    rows.append((float((g - g64).abs().max()) / max(float(g64.abs().max()), 1e-30), k))
rows.sort(reverse=True)
print(sys.argv[1] if len(sys.argv) > 1 else "", "worst vs branch-consistent fp64 oracle:", rows[:4])
