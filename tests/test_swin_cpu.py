"""CPU checks of the SwinUNETR oracle (oracle/swin_oracle.py) and of the
engine-side module tree.  PARITY UNPINNED: MONAI (the algorithm's home) is
absent offline and the reference holds no fixture for this model, so these
tests pin the restatement's internal conventions only: MONAI's state-dict
names/shapes, the relative-position index, the legacy PatchMerging order, the
zero-padding-after-norm1 attention semantics, and the Lit loss formula."""
import itertools

import pytest
import torch
import torch.nn.functional as F

from oracle import swin_oracle as S
from innovative3D.weightgen import synth_state


def test_registry_module_tree_matches_oracle_names():
    from innovative3D.config import variant
    lit = variant("SwinUNETR")[1]()
    # build_class drops window_size (not a LitSwinUNETR_Published kwarg) -> MONAI's 7
    assert lit.model.model.window == 7
    assert lit.hparams.include_bg_in_dice is False and lit.hparams.ce_weight == 0.5
    sd = lit.state_dict()
    shp = S.param_shapes(S.SwinCfg(num_classes=13), prefix="model.model.")
    keys = [k for k in sd if not k.endswith("relative_position_index")]
    assert keys == list(shp)
    assert all(tuple(sd[k].shape) == shp[k] for k in shp)
    for k, s in S.buffer_shapes(S.SwinCfg(), prefix="model.model.").items():
        assert torch.equal(sd[k], S.rel_index(7)) and tuple(sd[k].shape) == s


def test_rel_index_definition():
    w = 3
    idx = S.rel_index(w)
    coords = list(itertools.product(range(w), repeat=3))
    for i, ci in enumerate(coords):
        for j, cj in enumerate(coords):
            r = [a - b + w - 1 for a, b in zip(ci, cj)]
            assert idx[i, j] == (r[0] * (2 * w - 1) + r[1]) * (2 * w - 1) + r[2]


def test_merge_legacy_order():
    C = 2
    x = torch.arange(2 * 2 * 2 * C, dtype=torch.float64).view(1, 2, 2, 2, C)
    P = {"m.norm.weight": torch.ones(8 * C, dtype=torch.float64),
         "m.norm.bias": torch.zeros(8 * C, dtype=torch.float64),
         "m.reduction.weight": torch.eye(8 * C, dtype=torch.float64)}
    y = S._merge(P, "m.", x).view(8, C)
    cat = torch.stack([x[0, a, b, c] for a, b, c in S.STAGE_MERGE_ORDER])
    ref = F.layer_norm(cat.reshape(-1), (8 * C,)).view(8, C)
    assert torch.allclose(y, ref)
    # the quirk: slots 2/5 and 3/6 repeat, (1,1,0) and (0,1,1) never appear
    assert S.STAGE_MERGE_ORDER[2] == S.STAGE_MERGE_ORDER[5] == (0, 1, 0)
    assert S.STAGE_MERGE_ORDER[3] == S.STAGE_MERGE_ORDER[6] == (0, 0, 1)
    assert (1, 1, 0) not in S.STAGE_MERGE_ORDER and (0, 1, 1) not in S.STAGE_MERGE_ORDER


def test_window_attention_brute_force():
    """_window_attention vs a per-window loop: zero tokens padded after norm1
    take part as keys/values (k, v = qkv bias), outputs cropped."""
    torch.manual_seed(0)
    C, nh, w = 8, 2, 3
    x = torch.randn(1, 4, 5, 3, C, dtype=torch.float64)
    P = {"a.qkv.weight": torch.randn(3 * C, C, dtype=torch.float64) * 0.3,
         "a.qkv.bias": torch.randn(3 * C, dtype=torch.float64),
         "a.proj.weight": torch.randn(C, C, dtype=torch.float64) * 0.3,
         "a.proj.bias": torch.randn(C, dtype=torch.float64),
         "a.relative_position_bias_table": torch.randn((2 * w - 1) ** 3, nh, dtype=torch.float64)}
    ridx = S.rel_index(w)
    out = S._window_attention(P, "a.", x, nh, w, ridx)
    hd = C // nh
    ref = torch.zeros_like(x)
    xp = F.pad(x, (0, 0, 0, 0, 0, 1, 0, 2))  # -> 6 x 6 x 3
    for wd, wh in itertools.product(range(2), range(2)):
        toks = [(wd * 3 + a, wh * 3 + b, c) for a, b, c in itertools.product(range(3), repeat=3)]
        X = torch.stack([xp[0, d, h, ww] for d, h, ww in toks])
        qkv = X @ P["a.qkv.weight"].T + P["a.qkv.bias"]
        o = torch.zeros(27, C, dtype=torch.float64)
        for h_ in range(nh):
            q = qkv[:, h_ * hd:(h_ + 1) * hd] * hd ** -0.5
            k = qkv[:, C + h_ * hd:C + (h_ + 1) * hd]
            v = qkv[:, 2 * C + h_ * hd:2 * C + (h_ + 1) * hd]
            a = q @ k.T + P["a.relative_position_bias_table"][ridx.reshape(-1), h_].view(27, 27)
            o[:, h_ * hd:(h_ + 1) * hd] = torch.softmax(a, -1) @ v
        o = o @ P["a.proj.weight"].T + P["a.proj.bias"]
        for t, (d, h, ww) in enumerate(toks):
            if d < 4 and h < 5:
                ref[0, d, h, ww] = o[t]
    assert torch.allclose(out, ref, atol=1e-12)


def test_lit_loss_formula():
    torch.manual_seed(1)
    K = 4
    lg = torch.randn(2, K, 3, 4, 5, dtype=torch.float64)
    y = torch.randint(0, K, (2, 3, 4, 5))
    y[0, 0, 0, :2] = 255
    cfg = S.SwinCfg(num_classes=K)
    p = torch.softmax(lg, 1)
    m = (y != 255).double()
    yl = torch.where(y == 255, torch.zeros_like(y), y)
    dice = []
    for b in range(2):
        for c in range(1, K):
            g = (yl[b] == c).double()
            I = (p[b, c] * m[b] * g).sum()
            den = (p[b, c] * m[b]).sum() + g.sum() + 1e-6
            dice.append(2 * I / den)
    ce = F.cross_entropy(lg, y, ignore_index=255)
    ref = 0.5 * (1 - torch.stack(dice).mean()) + 0.5 * ce
    assert torch.allclose(S.lit_loss(lg, y, cfg), ref)


def test_oracle_fp32_vs_fp64_small():
    cfg = S.SwinCfg(num_classes=5)
    st = synth_state(list(S.param_shapes(cfg).items()), seed=1)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(1, 1, 32, 32, 64, generator=g)
    y = torch.randint(0, 5, (1, 32, 32, 64), generator=g)
    out = {}
    for dt in (torch.float64, torch.float32):
        P = S.params_from_state(st, dtype=dt)
        out[dt] = S.fwd_bwd(P, x, y, cfg)
    assert float((out[torch.float32][0].double() - out[torch.float64][0]).abs().max()) < 1e-4


def test_oracle_rejects_bad_sizes():
    cfg = S.SwinCfg(num_classes=3)
    P = S.params_from_state(synth_state(list(S.param_shapes(cfg).items()), seed=0))
    with pytest.raises(ValueError):
        S.forward(P, torch.randn(1, 1, 32, 32, 48), cfg)
