"""Use pytorch_lightning when it is installed (reference pins 2.6.1,
requirements.txt:70); otherwise a minimal stand-in with the same surface the
SPFF modules use (``save_hyperparameters``, ``hparams``, ``log``,
``trainer``).  Lightning drives the loop in the reference (train.py:1486-1516);
it is not part of the hot path."""
from __future__ import annotations

import types

import torch.nn as nn

try:  # pragma: no cover - depends on the environment
    import pytorch_lightning as pl  # type: ignore
    HAVE_LIGHTNING = True
except Exception:  # noqa: BLE001
    HAVE_LIGHTNING = False

    class AttributeDict(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

    class LightningModule(nn.Module):
        """nn.Module with Lightning's hyper-parameter and logging surface."""

        trainer = None

        def save_hyperparameters(self, *args, **kwargs):
            hp = AttributeDict()
            for a in args:
                if isinstance(a, dict):
                    hp.update(a)
            hp.update(kwargs)
            self.hparams = hp

        def log(self, name, value, *args, **kwargs):
            if not hasattr(self, "logged_metrics"):
                self.logged_metrics = {}
            self.logged_metrics[name] = value

    def seed_everything(seed=None, workers=False):
        import random

        import numpy as np
        import torch
        if seed is None:
            seed = 0
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
        return seed

    pl = types.SimpleNamespace(LightningModule=LightningModule, seed_everything=seed_everything,
                               AttributeDict=AttributeDict)

__all__ = ["pl", "HAVE_LIGHTNING"]
