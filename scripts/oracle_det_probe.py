#!/usr/bin/env python3
"""Run-to-run determinism of the fp64 oracle evaluated by PyTorch on the GPU at the
registry test's shape (1 x 1 x 5 x 512^2, K = 13, base 32): the oracle step is run
REPS times; every conv_in_lrelu output, pool output and parameter gradient is compared
with the first run's (max |diff| / max |ref|).  Test infrastructure (diagnostics only).

    python scripts/oracle_det_probe.py [REPS] [B C D H W]"""
import pathlib
import sys

import torch
import torch.nn.functional as F

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "spff-unet-spcct_amd")]
from oracle import spff_oracle as O  # noqa: E402
import innovative3D.models as M  # noqa: E402
from innovative3D.synthetic import synthetic_batch  # noqa: E402
from innovative3D.weightgen import synth_state  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
shape = tuple(int(a) for a in sys.argv[2:7]) if len(sys.argv) > 6 else (1, 1, 5, 512, 512)
K = 13
core = M.build_spct_energyfilm_fourier(num_classes=K, base=32, in_channels=shape[1])
for b in core._blocks():
    b.fgate._ensure_mask(shape[2], "cpu")
st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=0)
x, y = synthetic_batch(*shape, num_classes=K, ignore_frac=0.01, seed=6)
cfg = O.SpffCfg(in_ch=shape[1], num_classes=K, base=32)

rec = {}
orig_conv, orig_pool = O.conv_in_lrelu, O.maxpool


def _grad_hook(key):
    def h(g):
        rec[key] = g.detach().clone()
    return h


def conv_rec(P, pre, t, ksd):
    out = orig_conv(P, pre, t, ksd)
    rec[f"act {pre}"] = out.detach().clone()
    out.register_hook(_grad_hook(f"dact {pre}"))
    return out


npool = [0]


def pool_rec(t):
    out = orig_pool(t)
    rec[f"pool{npool[0] % 3 + 1}"] = out.detach().clone()
    out.register_hook(_grad_hook(f"dpool{npool[0] % 3 + 1}"))
    npool[0] += 1
    return out


O.conv_in_lrelu, O.maxpool = conv_rec, pool_rec


def _wrap(name):
    fn = getattr(O, name)

    def w(*a, **k):
        out = fn(*a, **k)
        pre = next((v for v in a if isinstance(v, str)), "")
        key = f"{name} {pre} #{len(rec)}"
        rec[key] = out.detach().clone()
        out.register_hook(_grad_hook("d_out " + key))
        return out
    setattr(O, name, w)


for _n in ("energy_film", "fourier_gate", "spectral_se", "se_channel", "_cat"):
    _wrap(_n)
if "SPFF_DET" in __import__("os").environ:
    torch.use_deterministic_algorithms(True)
    print("deterministic algorithms on", flush=True)
if "SPFF_HOST_FFT" in __import__("os").environ:
    _rfft, _irfft = torch.fft.rfft, torch.fft.irfft
    torch.fft.rfft = lambda t, *a, **k: _rfft(t.cpu(), *a, **k).to(t.device)
    torch.fft.irfft = lambda t, *a, **k: _irfft(t.cpu(), *a, **k).to(t.device)
    print("FFTs on the host", flush=True)
first = None
for r in range(reps):
    rec.clear()
    npool[0] = 0
    P = O.params_from_state({k: v for k, v in st.items() if not k.endswith("._mask")},
                            dtype=torch.float64, device="cuda")
    logits, loss, _, _ = O.fwd_bwd(P, x.to("cuda", torch.float64), y.to("cuda"), cfg)
    torch.cuda.synchronize()
    cur = {k: v.cpu() for k, v in rec.items()}
    cur["logits"] = logits.cpu()
    cur.update({f"grad {k}": v.grad.detach().cpu() for k, v in P.items()})
    del P, logits
    torch.cuda.empty_cache()
    if first is None:
        first = cur
        print(f"run 0: loss {float(loss):.12f}, {len(cur)} records", flush=True)
        continue
    bad = []
    for k, v in cur.items():
        ref = first[k]
        d = float((v - ref).abs().max() / ref.abs().max().clamp_min(1e-300))
        l2 = float((v - ref).norm() / ref.norm().clamp_min(1e-300))
        if d > 1e-12:
            bad.append((d, l2, k))
    # largest first (insertion order listed only the early activation records),
    # then every parameter-gradient record that moved -- the oracle's own gradients
    bad.sort(reverse=True)
    print(f"run {r}: loss {float(loss):.12f}; {len(bad)} records differ from run 0 "
          f"(max|diff|/max|ref|, rel L2), largest first:", flush=True)
    for d, l2, k in bad[:14]:
        print(f"    {k:40s} {d:.3e}  {l2:.3e}", flush=True)
    grads = [b for b in bad if b[2].startswith("grad ")]
    print(f"  parameter-gradient records that differ: {len(grads)} of "
          f"{sum(1 for k in cur if k.startswith('grad '))}", flush=True)
    for d, l2, k in grads[:10]:
        print(f"    {k:40s} {d:.3e}  {l2:.3e}", flush=True)
