"""apply_unified_optimizer() -- mirror of innovative3D/unified_optimizer.py:5-60.

Rebinds ``configure_optimizers`` of every LightningModule class in
``innovative3D.models`` (Adam/AdamW + optional poly / cosine schedules) and,
with ``disable_lr_hooks``, turns ``setup`` / ``on_train_batch_start`` /
``on_train_batch_end`` into no-ops, exactly like the reference."""
from __future__ import annotations

import torch

from innovative3D.lightning_compat import pl


def apply_unified_optimizer(lr: float = 1e-4, opt_cls=torch.optim.Adam, betas=(0.9, 0.999),
                            weight_decay: float = 0.0, schedule: str = "constant",
                            poly_power: float = 0.9, disable_lr_hooks: bool = True):
    import innovative3D.models as M

    from innovative3D.optim import SPFFAdam, SPFFAdamW

    def _cfg(self):
        if opt_cls in (torch.optim.Adam, torch.optim.AdamW, SPFFAdam, SPFFAdamW):
            opt = opt_cls(self.parameters(), lr=lr, betas=betas, weight_decay=weight_decay)
        else:
            opt = opt_cls(self.parameters(), lr=lr)
        trainer = getattr(self, "trainer", None)
        if schedule == "poly":
            T = getattr(trainer, "estimated_stepping_batches", None)
            if not T:
                steps = int(getattr(trainer, "num_training_batches", 0) or 100)
                epochs = int(getattr(trainer, "max_epochs", 0) or 100)
                T = steps * epochs

            def poly_lambda(step_idx: int):
                frac = max(0.0, 1.0 - step_idx / float(max(1, T)))
                return frac ** float(poly_power)

            sch = torch.optim.lr_scheduler.LambdaLR(opt, lr_lambda=poly_lambda)
            return {"optimizer": opt, "lr_scheduler": {"scheduler": sch, "interval": "step"}}
        if schedule == "cosine":
            T_max = int(getattr(trainer, "max_epochs", 0) or 100)
            sch = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=T_max)
            return {"optimizer": opt, "lr_scheduler": {"scheduler": sch, "interval": "epoch"}}
        return opt

    for _, cls in vars(M).items():
        if isinstance(cls, type) and issubclass(cls, pl.LightningModule):
            if not hasattr(cls, "_orig_configure_optimizers"):
                cls._orig_configure_optimizers = cls.configure_optimizers
            cls.configure_optimizers = _cfg
            if disable_lr_hooks:
                for hook in ("on_train_batch_start", "on_train_batch_end", "setup"):
                    if hasattr(cls, hook):
                        if not hasattr(cls, f"_orig_{hook}"):
                            setattr(cls, f"_orig_{hook}", getattr(cls, hook))
                        setattr(cls, hook, lambda *a, **k: None)
