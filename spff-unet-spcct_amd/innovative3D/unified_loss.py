"""apply_unified_loss() -- mirror of innovative3D/unified_loss.py:114-144.

Rebinds training/validation/test steps of every LightningModule class in
``innovative3D.models`` (except BaseLitModel) to the CE + 0.5*hard-Dice loss
plus metric logging.  The loss and the confusion counts behind the metrics
come from one fused HIP kernel (helpers.ce_dice_with_confusion)."""
from __future__ import annotations

import innovative3D.models as models_mod
from innovative3D.config import IGNORE_INDEX, NUM_CLASSES
from innovative3D.helpers import ce_dice_with_confusion, metrics_from_confusion
from innovative3D.lightning_compat import pl
from innovative3D.models import _canonicalize_targets_2d, _canonicalize_targets_3d, _pick_first_if_seq


def _get_num_classes(self) -> int:
    return int(getattr(getattr(self, "hparams", object()), "num_classes", NUM_CLASSES))


def _unified_shared_step(self, batch, stage: str):
    """unified_loss.py:29-99: tuple outputs -> main head; 5-D logits -> 3D."""
    if isinstance(batch, (list, tuple)):
        imgs, lbls = batch
    elif isinstance(batch, dict):
        imgs, lbls = batch.get("image"), batch.get("label")
    else:
        imgs, lbls = batch
    imgs = _pick_first_if_seq(imgs)
    lbls = _pick_first_if_seq(lbls)
    logits = self(imgs)
    if isinstance(logits, (list, tuple)):
        logits = logits[0]
    nc = _get_num_classes(self)
    ign = int(getattr(getattr(self, "hparams", object()), "ignore_index", IGNORE_INDEX))
    if logits.ndim == 5:
        tgt = _canonicalize_targets_3d(lbls).to(logits.device).long()
    elif logits.ndim == 4:
        tgt = _canonicalize_targets_2d(lbls).to(logits.device).long()
    else:
        raise RuntimeError(f"Unexpected logits ndim {logits.ndim}; expected 4D or 5D.")
    loss, conf = ce_dice_with_confusion(logits, tgt, nc, ign)
    (_d, _s, _sp, macro_dice, macro_sens, macro_spec, micro_dice, micro_sens,
     micro_spec) = metrics_from_confusion(conf.cpu().numpy(), nc, int(tgt.numel()))
    self.log(f"{stage}_loss", loss, on_step=False, on_epoch=True, prog_bar=(stage == "train"),
             sync_dist=True)
    self.log(f"{stage}_macro_dice", macro_dice, on_step=False, on_epoch=True,
             prog_bar=(stage != "test"), sync_dist=True)
    for k, v in (("micro_dice", micro_dice), ("macro_sens", macro_sens), ("macro_spec", macro_spec),
                 ("micro_sens", micro_sens), ("micro_spec", micro_spec)):
        self.log(f"{stage}_{k}", v, on_step=False, on_epoch=True, prog_bar=True, sync_dist=True)
    return loss


def _training_step(self, batch, batch_idx):
    return _unified_shared_step(self, batch, "train")


def _validation_step(self, batch, batch_idx):
    return _unified_shared_step(self, batch, "val")


def _test_step(self, batch, batch_idx):
    return _unified_shared_step(self, batch, "test")


def apply_unified_loss():
    patched = []
    for name in dir(models_mod):
        obj = getattr(models_mod, name)
        if not isinstance(obj, type) or not issubclass(obj, pl.LightningModule):
            continue
        if name == "BaseLitModel":
            continue
        obj.training_step = _training_step
        obj.validation_step = _validation_step
        obj.test_step = _test_step
        patched.append(name)
    if not patched:
        print("[unified_loss] No LightningModule classes found to patch.")
    else:
        print(f"[unified_loss] Patched Lightning steps for: {', '.join(sorted(patched))}")
    return patched
