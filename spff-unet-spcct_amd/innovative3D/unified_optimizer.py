"""apply_unified_optimizer() -- the API of innovative3D/unified_optimizer.py:5-60.

Contract kept from the reference (same signature, same effect on the module):
every LightningModule subclass in ``innovative3D.models`` gets a new
``configure_optimizers`` that builds ``opt_cls`` over the module's parameters
and, for ``schedule`` "poly" / "cosine", wraps it in the reference's schedulers
(``LambdaLR`` stepped per batch with ``(1 - t/T) ** poly_power``, clamped at 0;
``CosineAnnealingLR(T_max = max_epochs or 100)`` stepped per epoch).  The
original method is kept once as ``_orig_configure_optimizers``; with
``disable_lr_hooks`` the per-batch LR hooks and ``setup`` become no-ops (their
originals kept as ``_orig_<hook>``).

Expressed here as a table of schedule builders.  The fused HIP Adam/AdamW
(``innovative3D.optim.SPFFAdam/SPFFAdamW``) take the betas / weight-decay
arguments like ``torch.optim.Adam/AdamW``; any other optimizer class gets
``lr`` only, as in the reference (unified_optimizer.py:17-20).
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import torch

from innovative3D.lightning_compat import pl

_LR_HOOKS = ("on_train_batch_start", "on_train_batch_end", "setup")


def _trainer_total_steps(trainer) -> int:
    """Total optimizer steps for the poly decay: Lightning's estimate when it has
    one, else num_training_batches x max_epochs with 100 standing in for either
    when unknown (reference unified_optimizer.py:25-29)."""
    est = getattr(trainer, "estimated_stepping_batches", None)
    if est:
        return est
    per_epoch = int(getattr(trainer, "num_training_batches", 0) or 100)
    n_epochs = int(getattr(trainer, "max_epochs", 0) or 100)
    return per_epoch * n_epochs


def _poly(opt, trainer, poly_power: float):
    horizon = float(max(1, _trainer_total_steps(trainer)))
    power = float(poly_power)

    def factor(t: int) -> float:
        remaining = 1.0 - t / horizon
        return (remaining if remaining > 0.0 else 0.0) ** power

    return torch.optim.lr_scheduler.LambdaLR(opt, lr_lambda=factor), "step"


def _cosine(opt, trainer, _poly_power: float):
    t_max = int(getattr(trainer, "max_epochs", 0) or 100)
    return torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=t_max), "epoch"


# schedule name -> builder(opt, trainer, poly_power) -> (scheduler, Lightning interval);
# "constant" (or any other name) returns the bare optimizer
SCHEDULES: Dict[str, Callable] = {"poly": _poly, "cosine": _cosine}


def _adam_family():
    from innovative3D.optim import SPFFAdam, SPFFAdamW
    return (torch.optim.Adam, torch.optim.AdamW, SPFFAdam, SPFFAdamW)


def build_optimizer(params, lr: float, opt_cls, betas, weight_decay: float):
    if opt_cls in _adam_family():
        return opt_cls(params, lr=lr, betas=betas, weight_decay=weight_decay)
    return opt_cls(params, lr=lr)


def make_configure_optimizers(lr: float = 1e-4, opt_cls=torch.optim.Adam, betas=(0.9, 0.999),
                              weight_decay: float = 0.0, schedule: str = "constant",
                              poly_power: float = 0.9) -> Callable:
    """The ``configure_optimizers`` method that apply_unified_optimizer installs."""
    builder: Optional[Callable] = SCHEDULES.get(schedule)

    def configure_optimizers(self):
        opt = build_optimizer(self.parameters(), lr, opt_cls, betas, weight_decay)
        if builder is None:
            return opt
        sched, interval = builder(opt, getattr(self, "trainer", None), poly_power)
        return {"optimizer": opt, "lr_scheduler": {"scheduler": sched, "interval": interval}}

    return configure_optimizers


def _noop(*_a, **_k):
    return None


def _patch(cls, attr: str, new) -> None:
    """Replace cls.attr, remembering the first original as cls._orig_<attr>."""
    keep = f"_orig_{attr}"
    if not hasattr(cls, keep):
        setattr(cls, keep, getattr(cls, attr))
    setattr(cls, attr, new)


def apply_unified_optimizer(lr: float = 1e-4, opt_cls=torch.optim.Adam, betas=(0.9, 0.999),
                            weight_decay: float = 0.0, schedule: str = "constant",
                            poly_power: float = 0.9, disable_lr_hooks: bool = True):
    import innovative3D.models as M

    method = make_configure_optimizers(lr, opt_cls, betas, weight_decay, schedule, poly_power)
    lit_classes = [obj for obj in vars(M).values()
                   if isinstance(obj, type) and issubclass(obj, pl.LightningModule)]
    for cls in lit_classes:
        _patch(cls, "configure_optimizers", method)
        if disable_lr_hooks:
            for hook in _LR_HOOKS:
                if hasattr(cls, hook):
                    _patch(cls, hook, _noop)
