"""Loss and metrics of the SPFF hot path (mirror of innovative3D/helpers.py).

* ``ce_plus_macro_dice_loss`` (helpers.py:797-803): one fused HIP kernel --
  softmax-CE with ignore_index, its gradient, the argmax confusion matrix and
  the hard macro-Dice term, all on the device (no host syncs).  As in the
  reference, the Dice term is a constant: the gradient is the CE gradient only.
* ``macro_dice_loss`` (helpers.py:782-795) and ``per_class_metrics_3d/2d``
  (helpers.py:668-725, 728-779): the confusion counts come from the HIP kernel
  (one device->host copy); the NaN / absent-class algebra runs on the host
  exactly as the reference does it.

Only ``ce_plus_macro_dice`` is on the SPFF path (config.LOSS_NAME is never read
by it); the other LOSS_REGISTRY entries are out of scope and raise.
"""
from __future__ import annotations

import warnings
from typing import Optional

import numpy as np
import torch

from . import _engine as E

__all__ = ["ce_plus_macro_dice_loss", "macro_dice_loss", "per_class_metrics_3d",
           "per_class_metrics_2d", "metrics_from_confusion", "ce_dice_with_confusion",
           "ce_dice_parts", "dice_loss_from_confusion_t",
           "LOSS_REGISTRY"]


def _logits_cl(logits: torch.Tensor) -> torch.Tensor:
    """[B,K,D,H,W] (or [B,K,H,W]) -> channel-last contiguous; free for the
    engine's channels_last_3d logits."""
    if logits.ndim == 4:
        logits = logits.unsqueeze(2)
    if logits.ndim != 5:
        raise ValueError(f"expected [B,K,D,H,W] logits, got {tuple(logits.shape)}")
    return logits.permute(0, 2, 3, 4, 1).contiguous()


class _CEDice(torch.autograd.Function):
    """Outputs (loss, conf, ce): loss = ce + 0.5 * hard-Dice term (out4[1]); conf
    [K, K+1] and the CE share ce (out4[0]) carry no gradient."""

    @staticmethod
    def forward(ctx, logits, labels, K, ignore_index, smooth, count_override):
        lcl = _logits_cl(logits)
        out4, dl, conf = E.ce_dice_forward(lcl, labels, K, ignore_index, smooth, count_override)
        ctx.dl = dl
        ctx.ndim = logits.ndim
        ce = out4[0]
        ctx.mark_non_differentiable(conf, ce)
        return out4[1], conf, ce

    @staticmethod
    def backward(ctx, g, _gconf=None, _gce=None):
        # scaled in place (no second logits-sized buffer: 7 GB at 5 x 512^3) and handed
        # out exactly once; a retained-graph second backward would see a scaled tensor
        dl = ctx.dl
        if dl is None:
            raise RuntimeError("ce_plus_macro_dice_loss: backward ran twice through the same "
                               "graph (retain_graph); recompute the loss for a second backward")
        ctx.dl = None
        E.scale_(dl, g.reshape(1))
        d = dl.permute(0, 4, 1, 2, 3)
        if ctx.ndim == 4:
            d = d.squeeze(2)
        return d, None, None, None, None, None


def ce_dice_parts(logits, labels, num_classes, ignore_index=255, smooth=1e-6,
                  count_override: Optional[torch.Tensor] = None):
    """(loss, conf[K, K+1], ce) on the device with no host sync: loss as
    ce_plus_macro_dice_loss (differentiable through the CE only, as in the
    reference), conf[pred, label] of the argmax, ce = the CE term (with
    ``count_override`` = the global valid count, this rank's share of it)."""
    E.require_device(logits, "ce_plus_macro_dice_loss")
    if labels.ndim == logits.ndim and labels.shape[1] == 1:
        labels = labels[:, 0]
    return _CEDice.apply(logits, labels, int(num_classes), int(ignore_index), float(smooth),
                         count_override)


def ce_dice_with_confusion(logits, labels, num_classes, ignore_index=255, smooth=1e-6,
                           count_override: Optional[torch.Tensor] = None):
    """(loss, conf[K, K+1]) -- loss as ce_plus_macro_dice_loss; conf[pred, label]."""
    loss, conf, _ce = ce_dice_parts(logits, labels, num_classes, ignore_index, smooth,
                                    count_override)
    return loss, conf


def ce_plus_macro_dice_loss(logits, labels, num_classes, ignore_index=255, smooth=1e-6):
    """F.cross_entropy(ignore_index) + 0.5 * macro_dice_loss (helpers.py:797-803)."""
    loss, _conf = ce_dice_with_confusion(logits, labels, num_classes, ignore_index, smooth)
    return loss


def _conf_np(logits, labels, num_classes, ignore_index):
    conf = E.confusion(_logits_cl(logits.detach()), labels, int(num_classes), ignore_index)
    return conf.cpu().numpy()


def macro_dice_loss(logits, labels, num_classes, ignore_index=255, smooth=1e-6):
    """1 - mean_{c>=1} hard Dice, plain mean (no NaN skipping), python float."""
    conf = _conf_np(logits, labels, num_classes, ignore_index)
    return dice_loss_from_confusion(conf, num_classes, smooth)


def dice_loss_from_confusion(conf, num_classes, smooth=1e-6):
    """macro_dice_loss (helpers.py:782-795) from confusion counts conf[pred, label]
    (a column K of out-of-range labels, if present, counts as fp only)."""
    K = int(num_classes)
    vals = []
    for c in range(1, K):
        tp = int(conf[c, c])
        fp = int(conf[c, :].sum()) - tp
        fn = int(conf[:K, c].sum()) - tp
        vals.append((2 * tp + smooth) / (2 * tp + fp + fn + smooth))
    return 1.0 - (float(np.mean(vals)) if vals else 1.0)


def dice_loss_from_confusion_t(conf: torch.Tensor, num_classes: int,
                               smooth: float = 1e-6) -> torch.Tensor:
    """dice_loss_from_confusion with torch ops on conf's device (fp64, no host sync).
    conf: [K, K+1] or [K, K] counts (int64 or exactly-integer fp64)."""
    K = int(num_classes)
    c = conf.to(torch.float64)
    if K < 2:
        return torch.zeros((), dtype=torch.float64, device=conf.device)
    tp = torch.diagonal(c[:, :K])[1:]
    fp = c[1:K, :].sum(1) - tp
    fn = c[:K, 1:K].sum(0) - tp
    return 1.0 - ((2 * tp + smooth) / (2 * tp + fp + fn + smooth)).mean()


def metrics_from_confusion(conf: np.ndarray, K: int, n_voxels: int, smooth: float = 1e-6):
    """helpers.py:668-725 on counts.  conf is [K, K+1] (column K: labels not in
    [0,K), which count as 'not class c' for every c).  Reference quirk kept:
    tn uses the masked pred_c/label_c, so ignored voxels are true negatives
    (helpers.py:689) -> n_voxels = ALL voxels of the batch."""
    conf = np.asarray(conf, dtype=np.int64)
    dice_l, sens_l, spec_l = [], [], []
    for c in range(K):
        tp = int(conf[c, c])
        fp = int(conf[c, :].sum()) - tp
        fn = int(conf[:K, c].sum()) - tp
        tn = int(n_voxels) - tp - fp - fn
        if (tp + fn) == 0 and fp == 0:
            dice = float("nan"); sens = float("nan")
        else:
            dice = (2 * tp + smooth) / (2 * tp + fp + fn + smooth)
            sens = (tp + smooth) / (tp + fn + smooth) if (tp + fn) > 0 else float("nan")
        spec = (tn + smooth) / (tn + fp + smooth) if (tn + fp) > 0 else float("nan")
        dice_l.append(dice); sens_l.append(sens); spec_l.append(spec)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", RuntimeWarning)
        nm = lambda v: float(np.nanmean(v[1:])) if len(v) > 1 else float("nan")  # noqa: E731
        macro_dice, macro_sens, macro_spec = nm(dice_l), nm(sens_l), nm(spec_l)
    tp_sum = sum(int(conf[c, c]) for c in range(1, K))
    fp_sum = sum(int(conf[c, :].sum()) - int(conf[c, c]) for c in range(1, K))
    fn_sum = sum(int(conf[:K, c].sum()) - int(conf[c, c]) for c in range(1, K))
    tn_sum = int(conf[0, 0])
    dd = 2 * tp_sum + fp_sum + fn_sum
    micro_dice = (2 * tp_sum + smooth) / (dd + smooth) if dd > 0 else float("nan")
    micro_sens = (tp_sum + smooth) / (tp_sum + fn_sum + smooth) if (tp_sum + fn_sum) > 0 else float("nan")
    micro_spec = (tn_sum + smooth) / (tn_sum + fp_sum + smooth) if (tn_sum + fp_sum) > 0 else float("nan")
    return (dice_l, sens_l, spec_l, macro_dice, macro_sens, macro_spec, micro_dice, micro_sens,
            micro_spec)


def per_class_metrics_3d(preds, labels, num_classes, smooth=1e-6, ignore_index=None):
    """Returns the reference 9-tuple (dice/sens/spec lists, macro_*, micro_*)."""
    conf = _conf_np(preds, labels, num_classes, ignore_index)
    return metrics_from_confusion(conf, int(num_classes), int(labels.numel()), smooth)


def per_class_metrics_2d(preds, labels, num_classes, smooth=1e-6, ignore_index=None):
    return per_class_metrics_3d(preds, labels, num_classes, smooth, ignore_index)


def _out_of_scope(name):
    def _f(*a, **k):
        raise NotImplementedError(f"loss '{name}' is not on the SPFF hot path (config.LOSS_NAME is "
                                  f"never read by it); only 'ce_plus_macro_dice' is implemented")
    return _f


LOSS_REGISTRY = {
    "ce_plus_macro_dice": lambda logits, labels, nc, ignore_index: ce_plus_macro_dice_loss(
        logits, labels, nc, ignore_index=ignore_index),
    "focal_plus_gradient": _out_of_scope("focal_plus_gradient"),
    "dice_ce_nnunet": _out_of_scope("dice_ce_nnunet"),
}


# ------------------------------------------------------------- data path ---
# helpers.py:125-211 / 280-289, device-side: see
# innovative3D/datasets.py and csrc/data.hip.
def is_pixel_in_ellipse(x, y, roi):
    """helpers.py:125-129."""
    cx, cy = roi[0] + roi[2] / 2, roi[1] + roi[3] / 2
    a, b = roi[2] / 2, roi[3] / 2
    return ((x - cx) ** 2) / (a * a) + ((y - cy) ** 2) / (b * b) <= 1


def generate_cumulative_grid_sizes(num_images, num_grid_sizes=10, cumulative_percentage=0.2):
    """helpers.py:280-289 (module-level random, same draws)."""
    import random
    per = int(num_images * cumulative_percentage)
    out = []
    for gs in range(1, num_grid_sizes + 1):
        out.extend([gs] * per)
    rem = num_images - len(out)
    if rem > 0:
        out.extend(random.choices(range(1, num_grid_sizes + 1), k=rem))
    random.shuffle(out)
    return out


def read_dicom_frames(path):
    """Decoded frames [n, h, w] of one DICOM file: ``pydicom.dcmread(path).pixel_array`` as
    helpers.py:190-191 when pydicom is installed, else the native reader (innovative3D/dicom.py:
    uncompressed transfer syntaxes; a compressed one raises NotImplementedError)."""
    try:
        import pydicom
    except ImportError:
        from .dicom import pixel_array
        return pixel_array(path)
    return pydicom.dcmread(path).pixel_array


def create_image_and_labels_for_dataset(cfg, num_frames, frames_reader=None, device=None):
    """helpers.py:132-211 on the device: every DICOM under cfg["dir"] -> frames resized to
    IMAGE_HEIGHT x IMAGE_WIDTH (antialiased bilinear, TF.resize) and the ellipse-ROI label
    map (later ROIs overwrite).  Returns (images [N,F,H,W] fp32, labels [N,F,H,W] int64) on
    the device.  A list of configs is concatenated, as in the reference."""
    import os
    from pathlib import Path
    from .config import IMAGE_HEIGHT, IMAGE_WIDTH, global_label_names
    if isinstance(cfg, (list, tuple)):
        parts = [create_image_and_labels_for_dataset(c, num_frames, frames_reader, device)
                 for c in cfg]
        return torch.cat([p[0] for p in parts]), torch.cat([p[1] for p in parts])
    dev = device or torch.device("cuda")
    folder = os.path.expanduser(os.path.expandvars(str(Path(cfg["dir"]).resolve())))
    if not os.path.isdir(folder):
        raise FileNotFoundError(f"Images folder not found or not a directory: {folder}")
    paths = []
    for root, _, files in os.walk(folder):
        paths += [os.path.join(root, f) for f in files if f.lower().endswith((".dcm", ".dicom"))]
    if not paths:
        raise FileNotFoundError(f"No DICOM files (.dcm/.dicom) found under: {folder}")
    sx, sy = IMAGE_WIDTH / 1300.0, IMAGE_HEIGHT / 1300.0
    ox, oy = cfg["offset"]
    rois = []
    for (x, y, w, h, lab_str) in cfg["original_rois"]:
        lab = next((i for i, n in global_label_names.items() if n == lab_str), 0)
        rois.append((int((x + ox) * sx), int((y + oy) * sy), int(w * sx), int(h * sy), lab))
    rois_t = torch.tensor(rois, dtype=torch.int32).reshape(-1, 5).to(dev)
    reader = frames_reader or read_dicom_frames
    imgs, lbls = [], []
    for fn in paths:
        frames = np.asarray(reader(fn))
        n = min(frames.shape[0], num_frames)
        fr = torch.from_numpy(frames[:n].astype(np.float32)).to(dev)
        imgs.append(E.resize_bilinear_aa(fr, IMAGE_HEIGHT, IMAGE_WIDTH))
        lbls.append(E.rasterize_ellipses(rois_t, n, IMAGE_HEIGHT, IMAGE_WIDTH))
    return torch.stack(imgs), torch.stack(lbls)
