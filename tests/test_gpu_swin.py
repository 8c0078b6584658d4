"""SwinUNETR variant (BASELINE config 5) on the HIP engine vs the CPU oracle
(oracle/swin_oracle.py, MONAI 1.5.2 semantics restated).  PARITY UNPINNED:
MONAI is absent offline and the reference holds no fixture for this model, so
the oracle itself is pinned only by its own CPU tests (tests/test_swin_cpu.py).

Tolerances: logits within 1e-3 of the fp64 oracle (the north star's bar) and
identical argmax outside near-ties; loss within 1e-5 relative; every parameter
gradient within max(1e-3, 16 x the fp32 oracle's error) of max|g| per tensor,
against a kink-consistent oracle: the residual blocks' LeakyReLUs take the
engine's own sign pattern (its saved a1 / out tensors), since an input within
fp32 rounding of the kink may legitimately take either slope (1 vs 0.01)."""
import numpy as np
import pytest
import torch

from oracle import swin_oracle as S
from innovative3D.weightgen import synth_state
import innovative3D.models as M

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(B, D, H, W, K, seed):
    cfg = S.SwinCfg(num_classes=K)
    shp = S.param_shapes(cfg)
    st = synth_state(list(shp.items()), seed=seed)
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, 1, D, H, W, generator=g)
    y = torch.randint(0, K, (B, D, H, W), generator=g)
    y[torch.rand(B, D, H, W, generator=g) < 0.02] = 255
    return cfg, st, x, y


def _engine_model(st, K, mth):
    m = M.SwinUNETR(in_channels=1, out_channels=K, feature_size=12, depths=(1, 1, 1, 1),
                    num_heads=(1, 2, 4, 8), mlp_ratio=2.0)
    sd = m.state_dict()
    sd.update({k: torch.from_numpy(v) for k, v in st.items()})
    m.load_state_dict(sd, strict=True)
    m.math = mth
    return m.to(DEV)


@pytest.mark.parametrize("mth", ["f32", "bf16x6", "f16x3"])
@pytest.mark.parametrize("shape", [(2, 32, 64, 32), (1, 64, 64, 64), (1, 32, 32, 64)])
def test_swin_matches_oracle(shape, mth):
    B, D, H, W = shape
    K = 9
    cfg, st, x, y = _case(B, D, H, W, K, seed=3)
    m = _engine_model(st, K, mth)
    logits = m(x.to(DEV))
    loss = M._SwinLoss.apply(logits, y.to(DEV), K, 255, False, 0.5)
    loss.backward()
    torch.cuda.synchronize()
    lg = logits.detach().cpu().double()
    ref = {}
    S.ACT_MASKS = engine_act_masks(m, x.shape)
    try:
        for dt in (torch.float64, torch.float32):
            P = S.params_from_state(st, dtype=dt)
            rl, rloss = S.fwd_bwd(P, x, y, cfg)
            ref[dt] = (rl, rloss, {k: v.grad.double() for k, v in P.items()})
    finally:
        S.ACT_MASKS = None
    r64 = ref[torch.float64]
    err = float((lg - r64[0]).abs().max())
    print(f"{shape}/{mth}: max|dlogit| {err:.3e}  loss {float(loss):.7f} vs {float(r64[1]):.7f}")
    assert err <= 1e-3
    am, am_ref = lg.argmax(1), r64[0].argmax(1)
    top2 = r64[0].topk(2, dim=1).values
    ties = (top2[:, 0] - top2[:, 1]) < 2 * err
    assert not ((am != am_ref) & ~ties).any()
    assert abs(float(loss) - float(r64[1])) <= 1e-5 * abs(float(r64[1]))
    named = dict(m.named_parameters())
    rows, bad = [], []
    for k, g64 in r64[2].items():
        g = named[k].grad.detach().cpu().double()
        scale = max(float(g64.abs().max()), 1e-12)
        e = float((g - g64).abs().max()) / scale
        e32 = float((ref[torch.float32][2][k] - g64).abs().max()) / scale
        rows.append((e, e32, k))
        if e > max(1e-3, 16 * e32):
            bad.append(f"{k}: {e:.2e} (fp32 oracle {e32:.2e})")
    rows.sort(reverse=True)
    print("\n".join(f"  {k:60s} gpu {a:.2e}  fp32-oracle {b:.2e}" for a, b, k in rows[:8]))
    assert not bad, "; ".join(bad)


RB_LEVEL = {"encoder1.layer": 0, "encoder2.layer": 1, "encoder3.layer": 2, "encoder4.layer": 3,
            "encoder10.layer": 5, "decoder5.conv_block": 4, "decoder4.conv_block": 3,
            "decoder3.conv_block": 2, "decoder2.conv_block": 1, "decoder1.conv_block": 0}


def engine_act_masks(m, xshape):
    """Sign patterns of the residual blocks' LeakyReLU inputs as the engine saw
    them: sign(a1) and sign(out) (a LeakyReLU keeps the sign of its input)."""
    plan = m._plan(torch.empty(xshape, device=DEV))
    B, _, D, H, W = xshape
    out = {}
    for name, lvl in RB_LEVEL.items():
        for key, act in (("a1", "act1"), ("out", "act2")):
            t = plan.saved(f"{name}.{key}").cpu()
            C = t.shape[1]
            t = t.view(B, D >> lvl, H >> lvl, W >> lvl, C).permute(0, 4, 1, 2, 3)
            out[f"{name}.{act}"] = (t > 0).contiguous()
    return out


def test_swin_registry_forward_pads_to_32():
    """LitSwinUNETR_Published pads (replicate, centred) to a multiple of 32 and crops
    back (models.py:898-904): the registry layout [B, 1, 5, H, W]."""
    from innovative3D.config import variant
    lit = variant("SwinUNETR")[1]().to(DEV)
    x = torch.randn(1, 1, 5, 64, 64, device=DEV)
    with torch.no_grad():
        out = lit(x)
    assert tuple(out.shape) == (1, 13, 5, 64, 64)
    assert torch.isfinite(out).all()
