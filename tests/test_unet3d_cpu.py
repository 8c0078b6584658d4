"""3DUNet baseline variant (BASELINE config 3): the CPU oracle pinned to the
fixtures the reference itself produced (tests/golden/make_golden.py,
fxu3d_*), and the engine mirror's module tree / flat layouts.  CPU-only."""
import math

import numpy as np
import pytest
import torch

from _golden import load, unet3d_fixture_names, unet3d_state_of
from oracle import unet3d_oracle as U
from oracle import spff_oracle as O

NAMES = unet3d_fixture_names()


def cfg_of(meta):
    return U.UNet3DCfg(num_classes=meta["K"], base=meta["base"], in_ch=meta["in_ch"],
                       target_depth=meta["target_depth"])


def _prefix(meta):
    return "backbone." if meta.get("lit") else ""


@pytest.mark.parametrize("name", NAMES)
def test_unet3d_oracle_matches_reference(name):
    d = load(name)
    meta = d["meta"]
    cfg = cfg_of(meta)
    torch.set_num_threads(8)
    P, B = U.params_from_state(unet3d_state_of(d), prefix=_prefix(meta))
    x = torch.from_numpy(d["x"])
    y = torch.from_numpy(d["labels"])
    cw = torch.from_numpy(d["class_weights"]) if "class_weights" in d else None
    if meta.get("lit"):
        logits, loss = U.fwd_bwd(P, B, x, y, cfg, class_weights=cw)
    else:
        for t in P.values():
            t.grad = None
        lg = U.forward(P, B, x, cfg, True)
        loss = torch.nn.functional.cross_entropy(lg, y, ignore_index=255)
        loss.backward()
        logits = lg.detach()
    ref = d["logits"]
    err = float(np.abs(logits.numpy() - ref).max())
    assert err <= 2e-5, err
    assert torch.equal(logits.argmax(1), torch.from_numpy(ref).argmax(1))
    assert math.isclose(float(loss), float(d["loss"]), rel_tol=1e-5)
    met = O.per_class_metrics_3d(logits, y, meta["K"], ignore_index=255)
    np.testing.assert_allclose(np.array(met[0]), d["met_dice"], rtol=1e-12, equal_nan=True)
    np.testing.assert_allclose(np.array(met[3:]), d["met_scalars"], rtol=1e-12, equal_nan=True)
    # BatchNorm running statistics after the train-mode step (momentum 0.1, unbiased var)
    pre = _prefix(meta)
    for k in d:
        if k.startswith("bufafter/"):
            key = k[len("bufafter/"):]
            np.testing.assert_allclose(B[key[len(pre):]].numpy(), d[k], rtol=1e-5, atol=1e-6,
                                       err_msg=key)
    # gradients.  5e-4 of max|ref| + 2e-5 of the largest gradient entry of the model: the
    # fixture is one CPU's fp32 result and another CPU's oneDNN sums in another order
    # (observed on a second host: 1.3e-4 relative on the Cin=5 first-layer weight gradient,
    # 4.4e-7 absolute on a nearly cancelling BatchNorm bias gradient of max 2.8e-4; bitwise
    # equal on the host that wrote the fixtures).
    gmax = max(float(np.abs(d[k]).max()) for k in d
               if k.startswith("grad/") or k.startswith("gradhead/"))
    for k in d["param_names"]:
        k = str(k)
        g = P[k[len(pre):]].grad.numpy()
        if "grad/" + k in d:
            ref_g = d["grad/" + k]
            scale = max(1e-6, float(np.abs(ref_g).max()))
            assert float(np.abs(g - ref_g).max()) <= 5e-4 * scale + 2e-5 * gmax, k
        else:
            flat = g.reshape(-1)
            scale = max(1e-6, float(np.abs(d["gradhead/" + k]).max()))
            np.testing.assert_allclose(flat[:64], d["gradhead/" + k], atol=5e-4 * scale + 2e-5 * gmax)
            np.testing.assert_allclose(flat[-64:], d["gradtail/" + k], atol=5e-4 * scale + 2e-5 * gmax)
            s = d["gradsum/" + k]
            assert math.isclose(float(np.sqrt((flat.astype(np.float64) ** 2).sum())), float(s[1]),
                                rel_tol=1e-4, abs_tol=1e-9), k
    # eval mode on the updated running statistics
    with torch.no_grad():
        Pd = {k: v.detach() for k, v in P.items()}
        le = U.forward(Pd, B, x, cfg, False)
    assert float(np.abs(le.numpy() - d["logits_eval"]).max()) <= 2e-5


@pytest.mark.parametrize("name", NAMES)
def test_unet3d_layouts_match_reference_state_dict(name):
    """Module mirror, oracle and engine plan all use the reference's names/shapes/order."""
    import innovative3D.models as M
    from innovative3D import _engine as E
    d = load(name)
    meta = d["meta"]
    ref = d["state_shapes"]
    if meta.get("lit"):
        kw = {"class_weights": [1.0] * meta["K"]} if "class_weights" in d else {}
        m = M.LitCicek3DUNet_DepthAdapter_Published(num_classes=meta["K"], **kw)
    else:
        m = M.Cicek3DUNet(num_classes=meta["K"], base=meta["base"])
    sd = m.state_dict()
    assert list(sd.keys()) == list(ref.keys())
    assert all(tuple(sd[k].shape) == tuple(ref[k]) for k in sd)
    pre = _prefix(meta)
    cfg = cfg_of(meta)
    mine = U.param_shapes(cfg, prefix=pre)
    named = [(k, tuple(v.shape)) for k, v in m.named_parameters()]
    assert list(mine.items()) == named
    plan = E.UNet3DPlan(batch=1, in_ch=1, depth=d["x"].shape[2], height=32, width=32,
                        num_classes=meta["K"], base=meta["base"],
                        target_depth=meta["target_depth"])
    assert [(pre + n, s) for n, s, _o, _k in plan.params] == named
    offs = [o for _n, _s, o, _k in plan.params]
    assert offs == sorted(offs) and plan.nfloats == sum(int(np.prod(s)) for _n, s in named)
    bufs = [(pre + n) for n, _o, _k in plan.buffers]
    ref_bufs = [k for k in ref if k.endswith("running_mean") or k.endswith("running_var")]
    assert bufs == ref_bufs


def test_unet3d_registry_entry():
    from innovative3D import config as C
    import innovative3D.models as M
    name, factory, _dm, ck = C.variant("3DUNet")
    lit = factory()
    assert isinstance(lit, M.LitCicek3DUNet_DepthAdapter_Published)
    assert lit.target_depth == 16 and lit.class_weights is None and lit.dice_weight == 0.0
    opt = lit.configure_optimizers()
    assert isinstance(opt, torch.optim.SGD)
    g = opt.param_groups[0]
    assert (g["lr"], g["momentum"], g["nesterov"], g["weight_decay"]) == (1e-2, 0.99, False, 0.0)
    assert ck.name == "3DUNet"


def test_unet3d_plan_rejects_bad_shapes():
    from innovative3D import _engine as E
    with pytest.raises(E.SpffError, match="multiples of 16"):
        E.UNet3DPlan(batch=1, in_ch=1, depth=5, height=24, width=32, num_classes=13, base=32,
                     target_depth=16)
    with pytest.raises(E.SpffError):
        E.UNet3DPlan(batch=1, in_ch=1, depth=5, height=32, width=32, num_classes=129, base=32,
                     target_depth=16)   # K > SPFF_MAX_CLASSES
    with pytest.raises(E.SpffError):
        E.UNet3DPlan(batch=1, in_ch=1, depth=5, height=32, width=32, num_classes=13, base=12,
                     target_depth=16)   # base not a multiple of 8
    E.UNet3DPlan(batch=1, in_ch=1, depth=5, height=32, width=32, num_classes=40, base=24,
                 target_depth=16)


def test_unet3d_runs_only_on_device():
    import innovative3D.models as M
    from innovative3D import _engine as E
    m = M.Cicek3DUNet(num_classes=3, base=8)
    with pytest.raises(E.SpffError, match="no CPU fallback"):
        m(torch.zeros(1, 1, 16, 16, 16))
