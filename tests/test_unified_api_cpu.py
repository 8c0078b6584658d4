"""apply_unified_optimizer / apply_unified_loss API contract (CPU, no compute).

Reference: innovative3D/unified_optimizer.py:5-60 -- the patched
configure_optimizers returns the bare optimizer for "constant", and
{"optimizer", "lr_scheduler": {"scheduler", "interval"}} for "poly" (LambdaLR,
per step, (1 - t/T)^p clamped at 0) and "cosine" (CosineAnnealingLR(T_max =
max_epochs or 100), per epoch); originals are kept once as _orig_*."""
import types

import pytest
import torch

import innovative3D.models as M
from innovative3D.lightning_compat import pl
from innovative3D.unified_optimizer import apply_unified_optimizer


@pytest.fixture
def restore_lit_classes():
    lits = [c for c in vars(M).values() if isinstance(c, type) and issubclass(c, pl.LightningModule)]
    saved = {c: dict(vars(c)) for c in lits}
    yield lits
    for c, d in saved.items():
        for k in list(vars(c)):
            if k not in d:
                delattr(c, k)
        for k, v in d.items():
            if k.startswith("_orig_") or k in ("configure_optimizers", "on_train_batch_start",
                                               "on_train_batch_end", "setup"):
                setattr(c, k, v)


def _lit(trainer=None):
    m = M.LitSPCT_EFiLM_FourierGate(num_classes=9, base=8)
    if trainer is not None:
        object.__setattr__(m, "trainer", trainer)
    return m


def test_constant_returns_bare_adam(restore_lit_classes):
    apply_unified_optimizer(lr=3e-4, betas=(0.8, 0.99), weight_decay=0.01)
    opt = _lit().configure_optimizers()
    assert isinstance(opt, torch.optim.Adam)
    g = opt.param_groups[0]
    assert g["lr"] == 3e-4 and g["betas"] == (0.8, 0.99) and g["weight_decay"] == 0.01


def test_poly_schedule_shape_and_decay(restore_lit_classes):
    tr = types.SimpleNamespace(estimated_stepping_batches=10, num_training_batches=5, max_epochs=2)
    apply_unified_optimizer(lr=1.0, schedule="poly", poly_power=2.0)
    out = _lit(tr).configure_optimizers()
    assert set(out) == {"optimizer", "lr_scheduler"}
    assert set(out["lr_scheduler"]) == {"scheduler", "interval"}
    assert out["lr_scheduler"]["interval"] == "step"
    sch = out["lr_scheduler"]["scheduler"]
    assert isinstance(sch, torch.optim.lr_scheduler.LambdaLR)
    f = sch.lr_lambdas[0]
    assert f(0) == 1.0 and abs(f(5) - 0.25) < 1e-12 and f(10) == 0.0 and f(15) == 0.0


def test_poly_fallback_horizon(restore_lit_classes):
    # no estimate: T = num_training_batches * max_epochs, 100 for unknowns
    tr = types.SimpleNamespace(estimated_stepping_batches=None, num_training_batches=0,
                               max_epochs=3)
    apply_unified_optimizer(lr=1.0, schedule="poly", poly_power=1.0)
    f = _lit(tr).configure_optimizers()["lr_scheduler"]["scheduler"].lr_lambdas[0]
    assert abs(f(150) - 0.5) < 1e-12


def test_cosine_schedule(restore_lit_classes):
    tr = types.SimpleNamespace(max_epochs=None)
    apply_unified_optimizer(lr=1e-3, opt_cls=torch.optim.AdamW, schedule="cosine")
    out = _lit(tr).configure_optimizers()
    assert isinstance(out["optimizer"], torch.optim.AdamW)
    assert out["lr_scheduler"]["interval"] == "epoch"
    sch = out["lr_scheduler"]["scheduler"]
    assert isinstance(sch, torch.optim.lr_scheduler.CosineAnnealingLR) and sch.T_max == 100


def test_non_adam_gets_lr_only_and_hooks_disabled(restore_lit_classes):
    apply_unified_optimizer(lr=0.5, opt_cls=torch.optim.SGD)
    m = _lit()
    opt = m.configure_optimizers()
    assert isinstance(opt, torch.optim.SGD) and opt.param_groups[0]["lr"] == 0.5
    for cls in restore_lit_classes:
        assert hasattr(cls, "_orig_configure_optimizers")
        for hook in ("on_train_batch_start", "on_train_batch_end", "setup"):
            if hasattr(cls, hook):
                assert getattr(cls, hook)(None) is None
    # a second application keeps the FIRST original
    first = M.LitSPCT_EFiLM_FourierGate._orig_configure_optimizers
    apply_unified_optimizer(lr=0.1)
    assert M.LitSPCT_EFiLM_FourierGate._orig_configure_optimizers is first


def test_fused_adam_takes_betas(restore_lit_classes):
    from innovative3D.optim import SPFFAdam
    apply_unified_optimizer(lr=2e-4, opt_cls=SPFFAdam, betas=(0.5, 0.9))
    opt = _lit().configure_optimizers()
    assert isinstance(opt, SPFFAdam) and opt.param_groups[0]["betas"] == (0.5, 0.9)
