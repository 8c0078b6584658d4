"""SPFF-UNet model family -- drop-in mirror of innovative3D/models.py whose
forward/backward run on the MI355X HIP engine (libspff_hip.so).

The module tree (names, parameter shapes, registration order, the lazily
created and aliased FourierGate mask) is identical to the reference, so
state_dicts / checkpoints move between the two unchanged.  The nn.Conv3d /
nn.InstanceNorm3d / ... children are parameter containers only: their
forward is never called.  ``UNet3D_SpectralCore.forward`` hands the input and
one flat fp32 parameter buffer (the Parameters are views into it) to the
engine through a torch.autograd.Function; autograd receives the engine's
flat gradient back as per-parameter views.

Reference map (models.py): _SEChannelLite 600-609, _SpectralSE 611-614,
_conv3x3xk 616-618, _DoubleConvSpectral 620-625, UNet3D_SpectralCore 647-701,
_LitSPCT_Base 703-712, upgrade_spct_with_novel_blocks 1416-1446,
_DoubleConvSpectral_Novel 1448-1478, EnergyFiLM3D 1479-1512, FourierGate3D
1515-1544, build_spct_energyfilm_fourier 1547-1555, LitSPCT_* 1558-1607,
BaseLitModel 466-594.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _engine as E
from .config import BEST_LR, IGNORE_INDEX, NUM_CLASSES, NUM_FRAMES  # noqa: F401
from .helpers import (LOSS_REGISTRY, ce_plus_macro_dice_loss, ce_dice_with_confusion,  # noqa: F401
                      metrics_from_confusion, per_class_metrics_2d, per_class_metrics_3d)
from .lightning_compat import pl

# ----------------------------------------------------------------- utilities --


def _pick_first_if_seq(x):
    return x[0] if isinstance(x, (list, tuple)) else x


def _canonicalize_targets_2d(lbls):
    lbls = _pick_first_if_seq(lbls)
    if not torch.is_tensor(lbls):
        lbls = torch.as_tensor(lbls)
    if lbls.ndim == 4:
        lbls = lbls.max(dim=1).values
    elif lbls.ndim == 2:
        lbls = lbls.unsqueeze(0)
    return lbls.long()


def _canonicalize_targets_3d(lbls):
    """(B,1,F,H,W)/(B,F,H,W,1)/(F,H,W) -> (B,F,H,W) long (models.py:69-84)."""
    lbls = _pick_first_if_seq(lbls)
    if not torch.is_tensor(lbls):
        lbls = torch.as_tensor(lbls)
    if lbls.ndim == 5 and lbls.size(1) == 1:
        lbls = lbls[:, 0]
    if lbls.ndim == 5 and lbls.size(-1) == 1:
        lbls = lbls[..., 0]
    if lbls.ndim == 3:
        lbls = lbls.unsqueeze(0)
    assert lbls.ndim == 4, f"Need (B,F,H,W) labels, got {tuple(lbls.shape)}"
    return lbls.long()


def _next_mult(n: int, m: int = 16) -> int:
    return ((n + m - 1) // m) * m


def _pad_to_mult_3d(x: torch.Tensor, m: int = 16):
    """Replicate-pad D/H/W to multiples of m (models.py:109-120)."""
    B, C, D, H, W = x.shape
    Dn, Hn, Wn = _next_mult(D, m), _next_mult(H, m), _next_mult(W, m)
    pd, ph, pw = Dn - D, Hn - H, Wn - W
    if not (pd or ph or pw):
        return x, None
    x = F.pad(x, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2, pd // 2, pd - pd // 2),
              mode="replicate")
    return x, (D, H, W)


def _center_crop_to_3d(x: torch.Tensor, orig_dhw):
    if orig_dhw is None:
        return x
    D, H, W = orig_dhw
    _, _, Dn, Hn, Wn = x.shape
    sd, sh, sw = (Dn - D) // 2, (Hn - H) // 2, (Wn - W) // 2
    return x[:, :, sd:sd + D, sh:sh + H, sw:sw + W]


_pad_to_mult16_3d = lambda x, multiple=16: _pad_to_mult_3d(x, m=int(multiple))  # noqa: E731
_center_crop_3d = _center_crop_to_3d


def _norm3d(c: int, kind: str = "instance") -> nn.Module:
    if not (kind or "instance").lower().startswith("inst"):
        raise NotImplementedError("SPFF engine implements InstanceNorm3d(affine) only "
                                  "(models.py:168-173; SPFF never selects another norm)")
    return nn.InstanceNorm3d(c, affine=True, eps=1e-5)


def _act(kind: str = "lrelu") -> nn.Module:
    if not (kind or "lrelu").lower().startswith("lrel"):
        raise NotImplementedError("SPFF engine implements LeakyReLU(0.01) only (models.py:175-181)")
    return nn.LeakyReLU(1e-2, inplace=True)


def _conv3x3xk(cin, cout, ksd=1, bias=False):
    return nn.Conv3d(cin, cout, kernel_size=(ksd, 3, 3), padding=(ksd // 2, 1, 1), bias=bias)


# ------------------------------------------------------- parameter containers --
class _SEChannelLite(nn.Module):
    def __init__(self, c, r=16):
        super().__init__()
        h = max(4, c // r)
        self.pool = nn.AdaptiveAvgPool3d(1)
        self.fc = nn.Sequential(nn.Conv3d(c, h, 1, bias=True), nn.ReLU(inplace=True),
                                nn.Conv3d(h, c, 1, bias=True), nn.Sigmoid())


class _SpectralSE(nn.Module):
    pass


class _DoubleConvSpectral(nn.Module):
    def __init__(self, cin, cout, ksd=1, norm="instance", act="lrelu"):
        super().__init__()
        self.b1 = nn.Sequential(_conv3x3xk(cin, cout, ksd, bias=False), _norm3d(cout, norm), _act(act))
        self.b2 = nn.Sequential(_conv3x3xk(cout, cout, ksd, bias=False), _norm3d(cout, norm), _act(act))


class EnergyFiLM3D(nn.Module):
    """models.py:1479-1512 (parameter container; the engine computes it).  hidden 1..64,
    pe_dims 2..32 (include/spff.h spff_cfg.efilm_hidden / efilm_pe_dims), the same in every
    block of a network."""

    def __init__(self, channels: int, hidden: int = 32, pe_dims: int = 16):
        super().__init__()
        if not (1 <= int(hidden) <= 64 and 2 <= int(pe_dims) <= 32):
            raise NotImplementedError(
                f"EnergyFiLM3D(hidden={hidden}, pe_dims={pe_dims}): the engine supports hidden "
                "1..64 and pe_dims 2..32 (reference models.py:1484; pe_dims 1 makes the "
                "reference's own Conv1d raise); see INTEGRATION.md §2")
        self.channels = int(channels)
        self.hidden = int(hidden)
        self.pe_dims = int(pe_dims)
        self.mlp = nn.Sequential(nn.Conv1d(self.pe_dims, hidden, 1, bias=True), nn.ReLU(inplace=True),
                                 nn.Conv1d(hidden, 2 * self.channels, 1, bias=True))


class FourierGate3D(nn.Module):
    """Same lazy mask semantics as the reference (models.py:1527-1535):
    ``_mask``/``freq_mask`` (one tensor, two names) appear at the first forward.
    learn_phase=True multiplies the spectrum by (M + 0.01 i) (models.py:1538-1539), on the
    engine as an extra real circulant term (gates.hip phase_term)."""

    def __init__(self, learn_phase: bool = False):
        super().__init__()
        self.learn_phase = bool(learn_phase)
        self.mag_scale = nn.Parameter(torch.ones(1))
        self._mask = None

    def _ensure_mask(self, Fdim: int, device):
        L = Fdim // 2 + 1
        if (self._mask is None) or (self._mask.shape[2] != L):
            self._mask = nn.Parameter(torch.ones(1, 1, L, 1, 1, device=device,
                                                 dtype=self.mag_scale.dtype))
            self.register_parameter("freq_mask", self._mask)


class _DoubleConvSpectral_Novel(nn.Module):
    def __init__(self, cin, cout, ksd=1, norm="instance", act="lrelu", use_efilm: bool = False,
                 use_fouriergate: bool = False, use_moe: bool = False, moe_K: int = 3):
        super().__init__()
        if use_moe:
            # SpectralMoE3D is referenced but never defined in the reference (models.py:1464)
            raise NotImplementedError("use_moe: SpectralMoE3D does not exist in the reference")
        self.pre = nn.Sequential(_conv3x3xk(cin, cout, ksd, bias=False), _norm3d(cout, norm), _act(act))
        self.body = nn.Sequential(_conv3x3xk(cout, cout, ksd, bias=False), _norm3d(cout, norm), _act(act))
        self.efilm = EnergyFiLM3D(cout) if use_efilm else nn.Identity()
        self.fgate = FourierGate3D() if use_fouriergate else nn.Identity()


# --------------------------------------------------------- engine autograd op --
def _mark_covered(grad_hook, param_ids) -> None:
    """tell a GradBucketer which parameters' gradients it all-reduced (their flat
    gradient went through its buckets), so the caller reduces only the rest"""
    if grad_hook is not None and hasattr(grad_hook, "cover"):
        grad_hook.cover(param_ids)


class _SPFFFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, core, flat, *params):
        plan = core._plan
        logits_cl = plan.forward(x, flat)
        ctx.plan = plan
        ctx.gen = plan.generation
        ctx.flat = flat
        # a backward is pending on this workspace (E._alloc_workspace releases other
        # plans' workspaces on OOM, pending ones only as a last resort)
        plan._pending_gen = plan.generation if any(ctx.needs_input_grad) else None
        ctx.grad_hook = getattr(core, "grad_hook", None)
        ctx.param_ids = tuple(id(p) for p in params)
        ctx.slices = [(off, n, shape) for (_name, shape, off, n) in plan.params]
        return logits_cl.permute(0, 4, 1, 2, 3)

    @staticmethod
    def backward(ctx, g):
        plan = ctx.plan
        if plan.generation != ctx.gen:
            raise E.SpffError("SPFF engine: another forward ran on this model (or its cached workspace "
                              "was released for another plan's) before the backward "
                              "of this one; the engine keeps one forward's activations per model")
        g_cl = g.permute(0, 2, 3, 4, 1)
        if not g_cl.is_contiguous():
            g_cl = g_cl.contiguous()
        dflat = plan.backward(g_cl, ctx.flat, grad_hook=ctx.grad_hook)
        plan._pending_gen = None
        _mark_covered(ctx.grad_hook, ctx.param_ids)
        grads = [dflat[o:o + n].view(s) for (o, n, s) in ctx.slices]
        return (None, None, None, *grads)


# -------------------------------------------------------------------- core ----
class UNet3D_SpectralCore(nn.Module):
    """Depth-preserving 3-level UNet (models.py:647-701).  forward runs on the
    HIP engine; pool/upsample act in (H,W) only, so D is arbitrary while H, W
    must be multiples of 8."""

    def __init__(self, in_channels=1, num_classes=2, base=32, ksd=3, use_se=False,
                 use_specse=False, use_spatial=False, use_skip_gate=False, norm="instance",
                 act="lrelu"):
        super().__init__()
        if use_spatial or use_skip_gate:
            raise NotImplementedError("use_spatial/use_skip_gate are off on every SPCT registry "
                                      "entry (config.py:417-418) and not on the engine path")
        f = int(base)
        P = (1, 2, 2)
        self.in_channels, self.num_classes, self.base, self.ksd = int(in_channels), int(num_classes), f, int(ksd)
        self.use_se, self.use_specse = bool(use_se), bool(use_specse)
        self.enc1 = _DoubleConvSpectral(in_channels, f, ksd, norm, act)
        self.pool1 = nn.MaxPool3d(P)
        self.enc2 = _DoubleConvSpectral(f, 2 * f, ksd, norm, act)
        self.pool2 = nn.MaxPool3d(P)
        self.enc3 = _DoubleConvSpectral(2 * f, 4 * f, ksd, norm, act)
        self.pool3 = nn.MaxPool3d(P)
        self.bott = _DoubleConvSpectral(4 * f, 8 * f, ksd, norm, act)
        self.up3 = nn.ConvTranspose3d(8 * f, 4 * f, kernel_size=P, stride=P)
        self.dec3 = _DoubleConvSpectral(8 * f, 4 * f, ksd, norm, act)
        self.up2 = nn.ConvTranspose3d(4 * f, 2 * f, kernel_size=P, stride=P)
        self.dec2 = _DoubleConvSpectral(4 * f, 2 * f, ksd, norm, act)
        self.up1 = nn.ConvTranspose3d(2 * f, f, kernel_size=P, stride=P)
        self.dec1 = _DoubleConvSpectral(2 * f, f, ksd, norm, act)
        self.out = nn.Conv3d(f, num_classes, 1)
        self.se = nn.ModuleList([_SEChannelLite(c) if use_se else nn.Identity() for c in (f, 2 * f, 4 * f, 8 * f)])
        self.sp = nn.ModuleList([_SpectralSE() if use_specse else nn.Identity() for _ in range(4)])
        self.sa = nn.ModuleList([nn.Identity() for _ in range(4)])
        self.g3 = self.g2 = self.g1 = None
        self._plan = None
        self._flat = None
        self._infer_plan = None

    # ---- flags derived from the (possibly upgraded) module tree ----
    def _blocks(self):
        return [self.enc1, self.enc2, self.enc3, self.bott, self.dec3, self.dec2, self.dec1]

    def _flags(self) -> Tuple[bool, bool]:
        kinds = set()
        for b in self._blocks():
            if isinstance(b, _DoubleConvSpectral_Novel):
                kinds.add((isinstance(b.efilm, EnergyFiLM3D), isinstance(b.fgate, FourierGate3D)))
            else:
                kinds.add((False, False))
        if len(kinds) != 1:
            raise NotImplementedError("mixed block kinds; upgrade_spct_with_novel_blocks upgrades all")
        return next(iter(kinds))

    def _gate_settings(self) -> dict:
        """EnergyFiLM3D(hidden, pe_dims) / FourierGate3D(learn_phase) of the blocks (one
        setting for the whole network: include/spff.h spff_cfg)"""
        ef = {(b.efilm.hidden, b.efilm.pe_dims) for b in self._blocks()
              if isinstance(getattr(b, "efilm", None), EnergyFiLM3D)}
        ph = {b.fgate.learn_phase for b in self._blocks()
              if isinstance(getattr(b, "fgate", None), FourierGate3D)}
        if len(ef) > 1 or len(ph) > 1:
            raise NotImplementedError("EnergyFiLM3D(hidden, pe_dims) / FourierGate3D(learn_phase) "
                                      "must be the same in every block on the engine")
        h, pdim = next(iter(ef)) if ef else (32, 16)
        return {"efilm_hidden": h, "efilm_pe_dims": pdim,
                "fgate_learn_phase": bool(next(iter(ph))) if ph else False}

    def _engine_plan(self, x: torch.Tensor, tag: str):
        B, C, D, H, W = x.shape
        if C != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {C}")
        efilm, fgate = self._flags()
        # sharding (innovative3D.sharded): x is this rank's D-slab of a volume of
        # depth D * world (axis 0), or its H-slab of a volume of height H * world
        # (axis 1, the registry layout); the FourierGate acts on the full depth
        shard = E.shard_key(getattr(self, "shard", (1, 0)))
        if fgate:
            for b in self._blocks():
                b.fgate._ensure_mask(D * (shard[0] if shard[2] == 0 else 1), x.device)
        plan = E.get_plan(batch=B, in_ch=C, depth=D, height=H, width=W,
                          num_classes=self.num_classes, base=self.base, ksd=self.ksd,
                          efilm=efilm, fgate=fgate, se=self.use_se, specse=self.use_specse,
                          device=x.device, math=getattr(self, "math", None), shard=shard,
                          memory=getattr(self, "memory", None),
                          owner=self, tag=tag, **self._gate_settings())
        if shard[0] > 1:
            coll = getattr(self, "shard_coll", None)
            if coll is None:
                raise E.SpffError("sharded module: set .shard_coll (innovative3D.sharded)")
            if getattr(plan, "coll_impl", None) is not coll:
                plan.set_coll(coll)
        return plan

    def _engine_params(self, plan) -> List[nn.Parameter]:
        named = dict(self.named_parameters(remove_duplicate=False))
        out = []
        for name, shape, _off, _n in plan.params:
            p = named.get(name)
            if p is None or tuple(p.shape) != tuple(shape):
                raise E.SpffError(f"parameter {name} {shape} missing or mis-shaped in the module")
            out.append(p)
        return out

    def _ensure_flat(self, plan, params, device) -> torch.Tensor:
        flat = self._flat
        ok = flat is not None and flat.device == device and flat.numel() == plan.nfloats
        if ok:
            base = flat.data_ptr()
            for p, (_name, _shape, off, _n) in zip(params, plan.params):
                if p.data_ptr() != base + 4 * off or p.dtype != torch.float32:
                    ok = False
                    break
        if ok:
            return flat
        flat = torch.empty(plan.nfloats, dtype=torch.float32, device=device)
        with torch.no_grad():
            for p, (_name, shape, off, n) in zip(params, plan.params):
                flat[off:off + n].copy_(p.detach().reshape(-1).to(device=device, dtype=torch.float32))
                p.data = flat[off:off + n].view(shape)
        self._flat = flat
        return flat

    def forward(self, x):
        x = _pick_first_if_seq(x)
        E.require_device(x, "UNet3D_SpectralCore.forward")
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        plan = self._engine_plan(x, "train" if need_grad else "infer")
        params = self._engine_params(plan)
        flat = self._ensure_flat(plan, params, x.device)
        if need_grad:
            self._plan = plan
            return _SPFFFunction.apply(x.float(), self, flat, *params)
        logits_cl = plan.forward(x.float(), flat)
        return logits_cl.permute(0, 4, 1, 2, 3)


def upgrade_spct_with_novel_blocks(m: nn.Module, use_efilm: bool = True, use_fouriergate: bool = True,
                                   use_moe: bool = False, moe_K: int = 3):
    """models.py:1416-1446: replace every _DoubleConvSpectral by the novel block."""
    for name, child in list(m.named_children()):
        if isinstance(child, _DoubleConvSpectral):
            conv1, conv2 = child.b1[0], child.b2[0]
            new_block = _DoubleConvSpectral_Novel(int(conv1.in_channels), int(conv2.out_channels),
                                                  ksd=int(conv1.kernel_size[0]), use_efilm=use_efilm,
                                                  use_fouriergate=use_fouriergate, use_moe=use_moe,
                                                  moe_K=moe_K)
            setattr(m, name, new_block)
        else:
            upgrade_spct_with_novel_blocks(child, use_efilm, use_fouriergate, use_moe, moe_K)
    return m


def build_spct_energyfilm_fourier(num_classes=NUM_CLASSES, base=32, ksd=3, use_se=True, use_specse=True,
                                  use_spatial=False, use_skip_gate=False, in_channels=1, **kw):
    """models.py:1547-1555 (``in_channels`` added for the Cin=5 north-star layout)."""
    core = UNet3D_SpectralCore(in_channels=in_channels, num_classes=num_classes, base=base, ksd=ksd,
                               use_se=use_se, use_specse=use_specse, use_spatial=use_spatial,
                               use_skip_gate=use_skip_gate, **kw)
    return upgrade_spct_with_novel_blocks(core, use_efilm=True, use_fouriergate=True, use_moe=False)


# ----------------------------------------------------------- Lightning layer --
class BaseLitModel(pl.LightningModule):
    """models.py:466-594.  The loss is the fused HIP ce_plus_macro_dice kernel;
    metrics come from its confusion matrix (one host copy instead of ~100
    .item() syncs).  The test-only sklearn PR/ROC block (models.py:510-584) is
    host-side analytics outside the hot path and is not reproduced."""

    def __init__(self, num_classes=NUM_CLASSES, lr=BEST_LR, is_3d=True, **kwargs):
        super().__init__()
        self.is_3d = bool(is_3d)
        self.save_hyperparameters({"num_classes": num_classes, "lr": float(lr), "is_3d": bool(is_3d),
                                   **kwargs})
        self.lambda_esc = float(kwargs.get("lambda_esc", 0.0))
        self.lambda_smooth = float(kwargs.get("lambda_smooth", 0.0))

    def _normalize_input(self, x):
        return _pick_first_if_seq(x)

    def forward(self, x):
        return self.model(self._normalize_input(x))

    def compute_loss(self, logits, labels):
        return ce_plus_macro_dice_loss(logits, labels, self.hparams.num_classes, ignore_index=IGNORE_INDEX)

    def _shared_step(self, batch, prefix):
        imgs, lbls = batch if isinstance(batch, (list, tuple)) else (batch["image"], batch["label"])
        imgs = _pick_first_if_seq(imgs)
        lbls = _pick_first_if_seq(lbls)
        if not self.is_3d:
            lbls = _canonicalize_targets_2d(lbls)
        logits = self(imgs)
        lbls = lbls.to(logits.device).long()
        K = int(self.hparams.num_classes)
        loss, conf = ce_dice_with_confusion(logits, lbls, K, IGNORE_INDEX)
        # per_class_metrics_3d(logits, lbls, K, ignore_index=IGNORE_INDEX) from the same counts
        (dice_list, sens_list, spec_list, macro_dice, macro_sens, macro_spec,
         micro_dice, micro_sens, micro_spec) = metrics_from_confusion(conf.cpu().numpy(), K,
                                                                      int(lbls.numel()))
        self.log(f"{prefix}_loss", loss, on_step=False, on_epoch=True, prog_bar=(prefix == "train"),
                 sync_dist=True)
        self.log(f"{prefix}_macro_dice", macro_dice, on_step=False, on_epoch=True,
                 prog_bar=(prefix != "test"), sync_dist=True)
        for k, v in (("micro_dice", micro_dice), ("macro_sens", macro_sens), ("macro_spec", macro_spec),
                     ("micro_sens", micro_sens), ("micro_spec", micro_spec)):
            self.log(f"{prefix}_{k}", v, on_step=False, on_epoch=True, prog_bar=True, sync_dist=True)
        for i, (d, s, sp) in enumerate(zip(dice_list, sens_list, spec_list)):
            self.log(f"{prefix}_dice_class_{i}", d, on_step=False, on_epoch=True, prog_bar=False, sync_dist=True)
            self.log(f"{prefix}_sens_class_{i}", s, on_step=False, on_epoch=True, prog_bar=False, sync_dist=True)
            self.log(f"{prefix}_spec_class_{i}", sp, on_step=False, on_epoch=True, prog_bar=False, sync_dist=True)
        return loss

    def training_step(self, batch, batch_idx, dataloader_idx=0):
        return self._shared_step(batch, "train")

    def validation_step(self, batch, batch_idx, dataloader_idx=0):
        return {"val_loss": self._shared_step(batch, "val")}

    def test_step(self, batch, batch_idx):
        return self._shared_step(batch, "test")

    def configure_optimizers(self):
        # SPFF_FUSED_ADAM=1: the engine's fused Adam (same arithmetic, one pass)
        if os.environ.get("SPFF_FUSED_ADAM", "0") == "1":
            from .optim import SPFFAdam
            opt = SPFFAdam(self.parameters(), lr=self.hparams.lr)
        else:
            opt = torch.optim.Adam(self.parameters(), lr=self.hparams.lr)
        sch = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="max", factor=0.5, patience=5)
        return {"optimizer": opt, "lr_scheduler": {"scheduler": sch, "monitor": "val_macro_dice"}}


class _LitSPCT_Base(BaseLitModel):
    def __init__(self, num_classes=NUM_CLASSES, lr=BEST_LR, pad_multiple: int = 16):
        super().__init__(num_classes=num_classes, lr=lr, is_3d=True)
        self._pad_multiple = int(pad_multiple)

    def forward(self, x):
        x = _pick_first_if_seq(x)
        if x.ndim == 4:
            x = x.unsqueeze(1)
        x_pad, orig = _pad_to_mult16_3d(x, multiple=self._pad_multiple)
        return _center_crop_3d(self.model(x_pad), orig)


class LitSPCT_EFiLM_FourierGate(BaseLitModel):
    """The north-star model: registry entry "SPFF-UNet" (config.py:423-428)."""

    def __init__(self, num_classes=NUM_CLASSES, lr=BEST_LR, base=32, ksd=3, use_se=True, use_specse=True,
                 use_spatial=False, use_skip_gate=False, **kw):
        super().__init__(num_classes=num_classes, lr=lr, is_3d=True)
        self.model = build_spct_energyfilm_fourier(num_classes=num_classes, base=base, ksd=ksd,
                                                   use_se=use_se, use_specse=use_specse,
                                                   use_spatial=use_spatial, use_skip_gate=use_skip_gate, **kw)


class LitSPCT_EnergyFiLM(BaseLitModel):
    def __init__(self, num_classes=NUM_CLASSES, lr=BEST_LR, base=32, ksd=3, use_se=True, use_specse=True,
                 use_spatial=False, use_skip_gate=False, in_channels=1, **kw):
        super().__init__(num_classes=num_classes, lr=lr, is_3d=True, **kw)
        core = UNet3D_SpectralCore(in_channels=in_channels, num_classes=num_classes, base=base, ksd=ksd,
                                   use_se=use_se, use_specse=use_specse, use_spatial=use_spatial,
                                   use_skip_gate=use_skip_gate)
        self.model = upgrade_spct_with_novel_blocks(core, use_efilm=True, use_fouriergate=False)


class LitSPCT_FourierGate(BaseLitModel):
    def __init__(self, num_classes=NUM_CLASSES, lr=BEST_LR, base=32, ksd=3, use_se=True, use_specse=True,
                 use_spatial=False, use_skip_gate=False, in_channels=1, **kw):
        super().__init__(num_classes=num_classes, lr=lr, is_3d=True, **kw)
        core = UNet3D_SpectralCore(in_channels=in_channels, num_classes=num_classes, base=base, ksd=ksd,
                                   use_se=use_se, use_specse=use_specse, use_spatial=use_spatial,
                                   use_skip_gate=use_skip_gate)
        self.model = upgrade_spct_with_novel_blocks(core, use_efilm=False, use_fouriergate=True)


class LitSPCT_SEspec(_LitSPCT_Base):
    """Channel-SE + Spectral-SE at all stages (models.py:1585-1592)."""

    def __init__(self, num_classes=NUM_CLASSES, lr=BEST_LR, base=32, pad_multiple=16):
        super().__init__(num_classes=num_classes, lr=lr, pad_multiple=pad_multiple)
        self.model = UNet3D_SpectralCore(in_channels=1, num_classes=num_classes, base=base, ksd=3,
                                         use_se=True, use_specse=True, use_spatial=False,
                                         use_skip_gate=False)


class LitSPCT_ControlUNet(BaseLitModel):
    def __init__(self, num_classes=NUM_CLASSES, lr=BEST_LR, base=32, ksd=3, use_se=False, use_specse=False,
                 use_spatial=False, use_skip_gate=False, in_channels=1, **kw):
        super().__init__(num_classes=num_classes, lr=lr, is_3d=True, **kw)
        self.model = UNet3D_SpectralCore(in_channels=in_channels, num_classes=num_classes, base=base,
                                         ksd=ksd, use_se=use_se, use_specse=use_specse,
                                         use_spatial=use_spatial, use_skip_gate=use_skip_gate)


# ============================================================================
# 3DUNet baseline variant (BASELINE config 3; registry entry "3DUNet",
# config.py:283-311): Cicek3DUNet (models.py:718-753) + the depth-adapter
# Lightning wrapper (models.py:756-853), on the engine's spff_unet3d plan.
# ============================================================================
class _UNet3DFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan, flat, bufs, training, grad_hook, *params):
        logits_cl = plan.forward(x, flat, bufs, training)
        ctx.plan, ctx.gen, ctx.flat, ctx.grad_hook = plan, plan.generation, flat, grad_hook
        # a backward is pending on this workspace (E._alloc_workspace releases other
        # plans' workspaces on OOM, pending ones only as a last resort)
        plan._pending_gen = plan.generation if any(ctx.needs_input_grad) else None
        ctx.param_ids = tuple(id(p) for p in params)
        ctx.slices = [(off, n, shape) for (_name, shape, off, n) in plan.params]
        return logits_cl.permute(0, 4, 1, 2, 3)

    @staticmethod
    def backward(ctx, g):
        plan = ctx.plan
        if plan.generation != ctx.gen:
            raise E.SpffError("3DUNet engine: another forward ran on this model before the "
                              "backward of this one; the engine keeps one forward's activations")
        g_cl = g.permute(0, 2, 3, 4, 1).contiguous()
        dflat = plan.backward(g_cl, ctx.flat, grad_hook=ctx.grad_hook)
        plan._pending_gen = None
        _mark_covered(ctx.grad_hook, ctx.param_ids)
        grads = [dflat[o:o + n].view(s) for (o, n, s) in ctx.slices]
        return (None, None, None, None, None, None, *grads)


class Cicek3DUNet(nn.Module):
    """models.py:718-753.  Same module tree / state-dict keys as the reference
    (enc1.0.weight, enc1.1.running_mean, ..., up4.weight, out.bias); the
    Conv3d / BatchNorm3d children are parameter containers and forward runs on
    the engine (BatchNorm in train mode: batch statistics + running-stat update;
    eval mode: running statistics).  D, H, W must be multiples of 16."""

    def __init__(self, num_classes: int, base: int = 32, use_bn: bool = True, in_channels: int = 1):
        super().__init__()
        if not use_bn:
            raise NotImplementedError("use_bn=False (conv bias + Identity norm) is not on the "
                                      "registry path (config.py:308 sets use_bn=True)")

        def block(ci, co):
            return nn.Sequential(
                nn.Conv3d(ci, co, 3, padding=1, bias=False), nn.BatchNorm3d(co), nn.ReLU(inplace=True),
                nn.Conv3d(co, co, 3, padding=1, bias=False), nn.BatchNorm3d(co), nn.ReLU(inplace=True),
            )
        self.num_classes, self.base, self.in_channels = int(num_classes), int(base), int(in_channels)
        self.enc1 = block(in_channels, base); self.pool1 = nn.MaxPool3d(2)  # noqa: E702
        self.enc2 = block(base, base * 2); self.pool2 = nn.MaxPool3d(2)  # noqa: E702
        self.enc3 = block(base * 2, base * 4); self.pool3 = nn.MaxPool3d(2)  # noqa: E702
        self.enc4 = block(base * 4, base * 8); self.pool4 = nn.MaxPool3d(2)  # noqa: E702
        self.bott = block(base * 8, base * 16)
        self.up4 = nn.ConvTranspose3d(base * 16, base * 8, 2, stride=2)
        self.dec4 = block(base * 8 + base * 8, base * 8)
        self.up3 = nn.ConvTranspose3d(base * 8, base * 4, 2, stride=2)
        self.dec3 = block(base * 4 + base * 4, base * 4)
        self.up2 = nn.ConvTranspose3d(base * 4, base * 2, 2, stride=2)
        self.dec2 = block(base * 2 + base * 2, base * 2)
        self.up1 = nn.ConvTranspose3d(base * 2, base, 2, stride=2)
        self.dec1 = block(base + base, base)
        self.out = nn.Conv3d(base, num_classes, 1)
        self._flat = None
        self._bufs = None

    def _bn_modules(self):
        return [m for m in self.modules() if isinstance(m, nn.BatchNorm3d)]

    def _check_bn(self):
        for m in self._bn_modules():
            if (m.momentum != 0.1 or m.eps != 1e-5 or not m.affine or not m.track_running_stats):
                raise NotImplementedError("engine BatchNorm3d: momentum=0.1, eps=1e-5, affine, "
                                          "track_running_stats (the nn.BatchNorm3d defaults)")

    def _plan(self, x, target_depth: int):
        B, C, D, H, W = x.shape
        if C != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {C}")
        return E.get_unet3d_plan(batch=B, in_ch=C, depth=D, height=H, width=W,
                                 num_classes=self.num_classes, base=self.base,
                                 target_depth=int(target_depth) if target_depth != D else 0,
                                 device=x.device, math=getattr(self, "math", None),
                                 owner=self)

    def _engine_params(self, plan):
        named = dict(self.named_parameters())
        out = []
        for name, shape, _off, _n in plan.params:
            p = named.get(name)
            if p is None or tuple(p.shape) != tuple(shape):
                raise E.SpffError(f"parameter {name} {shape} missing or mis-shaped in the module")
            out.append(p)
        return out

    def _ensure_flat(self, plan, params, device):
        flat = self._flat
        ok = flat is not None and flat.device == device and flat.numel() == plan.nfloats
        if ok:
            base = flat.data_ptr()
            ok = all(p.data_ptr() == base + 4 * off and p.dtype == torch.float32
                     for p, (_n, _s, off, _k) in zip(params, plan.params))
        if not ok:
            flat = torch.empty(plan.nfloats, dtype=torch.float32, device=device)
            with torch.no_grad():
                for p, (_name, shape, off, n) in zip(params, plan.params):
                    flat[off:off + n].copy_(p.detach().reshape(-1).to(device=device,
                                                                     dtype=torch.float32))
                    p.data = flat[off:off + n].view(shape)
            self._flat = flat
        return flat

    def _ensure_bufs(self, plan, device):
        named = dict(self.named_buffers())
        bufs = self._bufs
        ok = bufs is not None and bufs.device == device and bufs.numel() == plan.nbuf
        if ok:
            base = bufs.data_ptr()
            ok = all(named[n].data_ptr() == base + 4 * off and named[n].dtype == torch.float32
                     for n, off, _k in plan.buffers)
        if not ok:
            bufs = torch.empty(plan.nbuf, dtype=torch.float32, device=device)
            with torch.no_grad():
                for name, off, n in plan.buffers:
                    b = named[name]
                    bufs[off:off + n].copy_(b.detach().reshape(-1).to(device=device,
                                                                      dtype=torch.float32))
                    b.data = bufs[off:off + n].view(b.shape)
            self._bufs = bufs
            for m in self._bn_modules():  # keep num_batches_tracked next to its stats
                m.num_batches_tracked.data = m.num_batches_tracked.data.to(device)
        return bufs

    def run(self, x, target_depth: int = 0):
        """Forward with the depth adapter fused in (target_depth > 0 resamples D
        there and back, models.py:771-777); returns [B,K,D,H,W] logits."""
        x = _pick_first_if_seq(x)
        E.require_device(x, "Cicek3DUNet.forward")
        self._check_bn()
        plan = self._plan(x, target_depth)
        params = self._engine_params(plan)
        flat = self._ensure_flat(plan, params, x.device)
        bufs = self._ensure_bufs(plan, x.device)
        plan.workspace(x.device)
        # data parallelism with synchronised BatchNorm: ``self.sync_bn`` = a collective with
        # allreduce(t) / world over the group (innovative3D.distributed.SyncBNGroup); None:
        # per-replica statistics (DDP without SyncBN, the reference's Lightning default)
        sync = getattr(self, "sync_bn", None)
        if getattr(plan, "_sync_impl", None) is not sync:
            plan.set_sync_bn(sync)
            plan._sync_impl = sync
        training = bool(self.training)
        if training:
            with torch.no_grad():
                for m in self._bn_modules():
                    m.num_batches_tracked.add_(1)
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        if need_grad:
            return _UNet3DFunction.apply(x.float(), plan, flat, bufs, training,
                                         getattr(self, "grad_hook", None), *params)
        return plan.forward(x.float(), flat, bufs, training).permute(0, 4, 1, 2, 3)

    def forward(self, x):
        return self.run(x, 0)


class _WeightedCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, K, ignore_index, class_weights):
        lcl = logits.permute(0, 2, 3, 4, 1).contiguous()
        out4, dl, conf = E.weighted_ce_forward(lcl, labels, K, ignore_index, class_weights)
        ctx.dl = dl
        ctx.mark_non_differentiable(conf)
        return out4[0], conf

    @staticmethod
    def backward(ctx, g, _gconf=None):
        dl = ctx.dl
        E.scale_(dl, g.reshape(1))
        return dl.permute(0, 4, 1, 2, 3), None, None, None, None


class LitCicek3DUNet_DepthAdapter_Published(pl.LightningModule):
    """models.py:756-853 (registry "3DUNet", config.py:283-311): depth adapter
    (resample D -> target_depth -> backbone -> back, fused into the engine),
    weighted softmax CE with ignore_index on the fused HIP loss kernel (class
    weights optional; denominator max(N_valid, 1)), macro-Dice logging from its
    confusion counts, SGD(momentum) as configure_optimizers."""

    def __init__(self, num_classes: int, target_depth: int = 16,
                 lr: float = 1e-2, momentum: float = 0.99, nesterov: bool = False,
                 weight_decay: float = 0.0, ignore_index: Optional[int] = 255,
                 class_weights: Optional[List[float]] = None, voxel_weight_key: Optional[str] = None,
                 ce_weight: float = 1.0, dice_weight: float = 0.0, use_bn: bool = True,
                 include_bg_in_dice: bool = False, *args, **kwargs):
        super().__init__()
        self.save_hyperparameters({"num_classes": num_classes, "target_depth": target_depth,
                                   "lr": lr, "momentum": momentum, "nesterov": nesterov,
                                   "weight_decay": weight_decay, "ignore_index": ignore_index,
                                   "class_weights": class_weights,
                                   "voxel_weight_key": voxel_weight_key, "ce_weight": ce_weight,
                                   "dice_weight": dice_weight, "use_bn": use_bn,
                                   "include_bg_in_dice": include_bg_in_dice})
        self.backbone = Cicek3DUNet(num_classes=num_classes, base=32, use_bn=use_bn)
        self.target_depth = int(target_depth)
        if class_weights is not None:
            cw = np.asarray(class_weights, dtype="float32")
            assert cw.shape[0] == int(num_classes)
            self.register_buffer("class_weights", torch.from_numpy(cw), persistent=True)
        else:
            self.class_weights = None
        self.voxel_weight_key = voxel_weight_key
        self.ignore_index = ignore_index
        self.include_bg_in_dice = include_bg_in_dice
        self.ce_weight = float(ce_weight)
        self.dice_weight = float(dice_weight)

    def forward(self, x):
        return self.backbone.run(_pick_first_if_seq(x), self.target_depth)

    def _weighted_softmax_ce(self, logits, target, voxel_weights: Optional[torch.Tensor]):
        if target.ndim == 5 and target.shape[1] == 1:
            target = target[:, 0]
        if voxel_weights is not None:
            raise NotImplementedError("per-voxel CE weights (voxel_weight_key) are off on the "
                                      "registry path (config.py:297)")
        ign = self.ignore_index if self.ignore_index is not None else -1000
        loss, conf = _WeightedCE.apply(logits, target, int(self.hparams.num_classes), int(ign),
                                       getattr(self, "class_weights", None))
        self._last_conf = conf
        return loss

    def _dice_loss(self, logits, y, eps=1e-6):
        raise NotImplementedError("the soft-Dice term (dice_weight > 0) is off on the registry "
                                  "path (config.py:300: dice_weight=0.0)")

    def _loss_and_log(self, logits, y, stage: str, voxel_w: Optional[torch.Tensor],
                      log_metrics: bool = True):
        ce = self._weighted_softmax_ce(logits, y, voxel_w) * self.ce_weight
        loss = ce
        if self.dice_weight > 0.0:
            loss = loss + self._dice_loss(logits, y) * self.dice_weight
        self.log(f"{stage}_loss", loss, prog_bar=(stage == "train"), on_step=False, on_epoch=True,
                 sync_dist=True)
        if log_metrics:
            # per_class_metrics_3d(logits, tgt, K, ignore_index) from the argmax counts the
            # loss kernel already produced (ignore_index None <-> the loss's -1000: no label
            # equals either, so the counts are the same)
            tgt = _canonicalize_targets_3d(y)
            K = int(self.hparams.num_classes)
            met = metrics_from_confusion(self._last_conf.cpu().numpy(), K, int(tgt.numel()))
            self.log(f"{stage}_macro_dice", met[3], on_step=False, on_epoch=True, prog_bar=True,
                     sync_dist=True)
        return loss

    def _unpack(self, batch):
        if isinstance(batch, (list, tuple)):
            x, y = batch
            voxel_w = None
        else:
            x, y = batch["image"], batch["label"]
            voxel_w = batch.get(self.voxel_weight_key) if self.voxel_weight_key is not None else None
        return x, y, voxel_w

    def training_step(self, batch, _):
        x, y, vw = self._unpack(batch)
        logits = self(x)
        return self._loss_and_log(logits, y.to(logits.device), "train", voxel_w=vw)

    def validation_step(self, batch, _):
        x, y, vw = self._unpack(batch)
        logits = self(x)
        return self._loss_and_log(logits, y.to(logits.device), "val", voxel_w=vw, log_metrics=True)

    def test_step(self, batch, _):
        x, y, vw = self._unpack(batch)
        logits = self(x)
        return self._loss_and_log(logits, y.to(logits.device), "test", voxel_w=vw)

    def configure_optimizers(self):
        return torch.optim.SGD(self.parameters(), lr=self.hparams.lr,
                               momentum=self.hparams.momentum,
                               nesterov=bool(self.hparams.nesterov),
                               weight_decay=self.hparams.weight_decay)


# ============================================================================
# SwinUNETR variant (BASELINE config 5; registry "SwinUNETR", config.py:366-386):
# LitSwinUNETR_Published (models.py:880-982) around SwinUNETR_Published
# (models.py:858-878), i.e. MONAI 1.5.2 SwinUNETR, on the engine's spff_swin
# plan.  The module tree below only holds parameters under MONAI's state-dict
# names; forward runs on the HIP engine.  Parity unpinned (no MONAI offline):
# semantics in oracle/swin_oracle.py.
# ============================================================================
class _SwinFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, plan, flat, grad_hook, *params):
        logits_cl = plan.forward(x, flat)
        ctx.plan, ctx.gen, ctx.flat, ctx.grad_hook = plan, plan.generation, flat, grad_hook
        # a backward is pending on this workspace (E._alloc_workspace releases other
        # plans' workspaces on OOM, pending ones only as a last resort)
        plan._pending_gen = plan.generation if any(ctx.needs_input_grad) else None
        ctx.param_ids = tuple(id(p) for p in params)
        ctx.slices = [(off, n, shape) for (_name, shape, off, n) in plan.params]
        return logits_cl.permute(0, 4, 1, 2, 3)

    @staticmethod
    def backward(ctx, g):
        plan = ctx.plan
        if plan.generation != ctx.gen:
            raise E.SpffError("SwinUNETR engine: another forward ran on this model before the "
                              "backward of this one; the engine keeps one forward's activations")
        g_cl = g.permute(0, 2, 3, 4, 1).contiguous()
        dflat = plan.backward(g_cl, ctx.flat, grad_hook=ctx.grad_hook)
        plan._pending_gen = None
        _mark_covered(ctx.grad_hook, ctx.param_ids)
        grads = [dflat[o:o + n].view(s) for (o, n, s) in ctx.slices]
        return (None, None, None, None, *grads)


class _Holder(nn.Module):
    """Parameter container (MONAI module names; no forward)."""


def _conv_holder(conv: nn.Module) -> nn.Module:
    h = _Holder()
    h.conv = conv
    return h


def _res_block(ci: int, co: int) -> nn.Module:
    """MONAI UnetResBlock (conv1.conv, conv2.conv[, conv3.conv]; InstanceNorm3d
    without affine has no parameters)."""
    r = _Holder()
    r.conv1 = _conv_holder(nn.Conv3d(ci, co, 3, padding=1, bias=False))
    r.conv2 = _conv_holder(nn.Conv3d(co, co, 3, padding=1, bias=False))
    if ci != co:
        r.conv3 = _conv_holder(nn.Conv3d(ci, co, 1, bias=False))
    return r


class _WindowAttentionP(nn.Module):
    def __init__(self, dim: int, heads: int, window: int):
        super().__init__()
        self.relative_position_bias_table = nn.Parameter(
            torch.zeros((2 * window - 1) ** 3, heads))
        nn.init.trunc_normal_(self.relative_position_bias_table, std=0.02)
        c = torch.stack(torch.meshgrid(torch.arange(window), torch.arange(window),
                                       torch.arange(window), indexing="ij")).flatten(1)
        r = (c[:, :, None] - c[:, None, :]).permute(1, 2, 0) + (window - 1)
        idx = r[..., 0] * (2 * window - 1) ** 2 + r[..., 1] * (2 * window - 1) + r[..., 2]
        self.register_buffer("relative_position_index", idx)
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim)


class _SwinBlockP(nn.Module):
    def __init__(self, dim: int, heads: int, window: int, mlp_ratio: float):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim)
        self.attn = _WindowAttentionP(dim, heads, window)
        self.norm2 = nn.LayerNorm(dim)
        self.mlp = _Holder()
        self.mlp.linear1 = nn.Linear(dim, int(dim * mlp_ratio))
        self.mlp.linear2 = nn.Linear(int(dim * mlp_ratio), dim)


class _BasicLayerP(nn.Module):
    def __init__(self, dim: int, heads: int, window: int, mlp_ratio: float):
        super().__init__()
        self.blocks = nn.ModuleList([_SwinBlockP(dim, heads, window, mlp_ratio)])
        self.downsample = _Holder()
        self.downsample.reduction = nn.Linear(8 * dim, 2 * dim, bias=False)
        self.downsample.norm = nn.LayerNorm(8 * dim)


class SwinUNETR(nn.Module):
    """MONAI 1.5.2 SwinUNETR (patch_size 2, depths (1,1,1,1) -- the registry's --,
    normalize=True, res_block, InstanceNorm, downsample "merging", use_v2 False)
    with MONAI's parameter names; forward on the HIP engine (D, H, W multiples
    of 32, as MONAI's _check_input_size requires)."""

    def __init__(self, in_channels: int = 1, out_channels: int = 2, feature_size: int = 24,
                 depths=(2, 2, 2, 2), num_heads=(3, 6, 12, 24), window_size=7,
                 mlp_ratio: float = 4.0, qkv_bias: bool = True, norm_name="instance",
                 drop_rate: float = 0.0, attn_drop_rate: float = 0.0,
                 dropout_path_rate: float = 0.0, normalize: bool = True, use_checkpoint=False,
                 spatial_dims: int = 3, downsample="merging", use_v2: bool = False, **_):
        super().__init__()
        ws = window_size if isinstance(window_size, int) else int(window_size[0])
        if not isinstance(window_size, int) and len(set(window_size)) != 1:
            raise NotImplementedError("cubic windows only")
        if tuple(depths) != (1, 1, 1, 1):
            raise NotImplementedError("depths (1,1,1,1) only (the registry's, config.py:374)")
        if (not qkv_bias or not normalize or use_v2 or downsample != "merging" or spatial_dims != 3
                or str(norm_name).lower() != "instance"):
            raise NotImplementedError("the registry's SwinUNETR settings only (qkv_bias, normalize, "
                                      "merging, instance norm, 3D, use_v2=False)")
        if drop_rate or attn_drop_rate or dropout_path_rate:
            raise NotImplementedError("dropout / drop-path are 0 on the registry path")
        f = int(feature_size)
        self.in_channels, self.num_classes, self.feature_size = int(in_channels), int(out_channels), f
        self.window, self.num_heads, self.mlp_ratio = ws, tuple(int(h) for h in num_heads), float(mlp_ratio)
        self.swinViT = _Holder()
        self.swinViT.patch_embed = _Holder()
        self.swinViT.patch_embed.proj = nn.Conv3d(in_channels, f, 2, stride=2)
        for s in range(4):
            setattr(self.swinViT, f"layers{s + 1}",
                    nn.ModuleList([_BasicLayerP(f << s, self.num_heads[s], ws, mlp_ratio)]))
        self.encoder1 = _Holder(); self.encoder1.layer = _res_block(in_channels, f)  # noqa: E702
        self.encoder2 = _Holder(); self.encoder2.layer = _res_block(f, f)  # noqa: E702
        self.encoder3 = _Holder(); self.encoder3.layer = _res_block(2 * f, 2 * f)  # noqa: E702
        self.encoder4 = _Holder(); self.encoder4.layer = _res_block(4 * f, 4 * f)  # noqa: E702
        self.encoder10 = _Holder(); self.encoder10.layer = _res_block(16 * f, 16 * f)  # noqa: E702
        for name, ci, co in (("decoder5", 16 * f, 8 * f), ("decoder4", 8 * f, 4 * f),
                             ("decoder3", 4 * f, 2 * f), ("decoder2", 2 * f, f), ("decoder1", f, f)):
            d = _Holder()
            d.transp_conv = _conv_holder(nn.ConvTranspose3d(ci, co, 2, stride=2, bias=False))
            d.conv_block = _res_block(2 * co, co)
            setattr(self, name, d)
        self.out = _Holder()
        self.out.conv = _conv_holder(nn.Conv3d(f, out_channels, 1, bias=True))
        self._flat = None

    def _plan(self, x):
        B, C, D, H, W = x.shape
        if C != self.in_channels:
            raise ValueError(f"expected {self.in_channels} input channels, got {C}")
        if D % 32 or H % 32 or W % 32:
            raise ValueError(f"spatial dims {(D, H, W)} must be divisible by 2**5 = 32")
        return E.get_swin_plan(batch=B, in_ch=C, depth=D, height=H, width=W,
                               num_classes=self.num_classes, feature_size=self.feature_size,
                               window=self.window, heads=self.num_heads, mlp_ratio=self.mlp_ratio,
                               device=x.device, math=getattr(self, "math", None),
                               owner=self)

    def _engine_params(self, plan):
        named = dict(self.named_parameters())
        out = []
        for name, shape, _off, _n in plan.params:
            p = named.get(name)
            if p is None or tuple(p.shape) != tuple(shape):
                raise E.SpffError(f"parameter {name} {shape} missing or mis-shaped in the module")
            out.append(p)
        return out

    def _ensure_flat(self, plan, params, device):
        flat = self._flat
        ok = flat is not None and flat.device == device and flat.numel() == plan.nfloats
        if ok:
            base = flat.data_ptr()
            ok = all(p.data_ptr() == base + 4 * off and p.dtype == torch.float32
                     for p, (_n, _s, off, _k) in zip(params, plan.params))
        if not ok:
            flat = torch.empty(plan.nfloats, dtype=torch.float32, device=device)
            with torch.no_grad():
                for p, (_name, shape, off, n) in zip(params, plan.params):
                    flat[off:off + n].copy_(p.detach().reshape(-1).to(device=device,
                                                                     dtype=torch.float32))
                    p.data = flat[off:off + n].view(shape)
            self._flat = flat
        return flat

    def forward(self, x_in):
        E.require_device(x_in, "SwinUNETR.forward")
        plan = self._plan(x_in)
        params = self._engine_params(plan)
        flat = self._ensure_flat(plan, params, x_in.device)
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            return _SwinFunction.apply(x_in.float(), plan, flat, getattr(self, "grad_hook", None),
                                       *params)
        return plan.forward(x_in.float(), flat).permute(0, 4, 1, 2, 3)


class SwinUNETR_Published(nn.Module):
    """models.py:858-878: builds SwinUNETR with the kwargs MONAI 1.5.2 accepts
    (img_size dropped, drop_path_rate -> dropout_path_rate, spatial_dims=3)."""

    def __init__(self, num_classes, img_size=(96, 96, 96), in_channels=1, feature_size=48,
                 depths=(2, 2, 2, 2), num_heads=(3, 6, 12, 24), mlp_ratio=4.0, drop_rate=0.0,
                 attn_drop_rate=0.0, dropout_path_rate=0.0, use_checkpoint=False,
                 norm_name="instance", **kwargs):
        super().__init__()
        self.model = SwinUNETR(in_channels=in_channels, out_channels=num_classes,
                               feature_size=feature_size, depths=depths, num_heads=num_heads,
                               mlp_ratio=mlp_ratio, drop_rate=drop_rate,
                               attn_drop_rate=attn_drop_rate, dropout_path_rate=dropout_path_rate,
                               use_checkpoint=use_checkpoint, norm_name=norm_name, spatial_dims=3)

    def forward(self, x):
        return self.model(x)


class _SwinLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, K, ignore_index, include_bg, ce_weight):
        lcl = logits.permute(0, 2, 3, 4, 1).contiguous()
        out4, dl = E.swin_loss_forward(lcl, labels, K, ignore_index, include_bg, ce_weight)
        ctx.dl = dl
        return out4[1]

    @staticmethod
    def backward(ctx, g):
        dl = ctx.dl
        E.scale_(dl, g.reshape(1))
        return dl.permute(0, 4, 1, 2, 3), None, None, None, None, None


class LitSwinUNETR_Published(pl.LightningModule):
    """models.py:880-982 (registry "SwinUNETR"): pad to a multiple of 32 (replicate,
    centred) -> SwinUNETR -> crop; loss (1 - w) soft-Dice + w CE(ignore) on the
    fused HIP loss kernels; AdamW with linear warm-up + cosine decay."""

    def __init__(self, num_classes: int, img_size=(96, 96, 96), in_channels: int = 1,
                 feature_size: int = 48, depths=(2, 2, 2, 2), num_heads=(3, 6, 12, 24),
                 mlp_ratio: float = 4.0, drop_rate: float = 0.0, attn_drop_rate: float = 0.0,
                 dropout_path_rate: float = 0.0, use_checkpoint: bool = False,
                 norm_name: str = "instance", lr: float = 1e-4, weight_decay: float = 1e-2,
                 warmup_epochs: int = 5, use_ce_alongside_dice: bool = True,
                 ce_weight: float = 0.5, ignore_index: Optional[int] = IGNORE_INDEX,
                 include_bg_in_dice: bool = True):
        super().__init__()
        self.save_hyperparameters({
            "num_classes": num_classes, "img_size": img_size, "in_channels": in_channels,
            "feature_size": feature_size, "depths": depths, "num_heads": num_heads,
            "mlp_ratio": mlp_ratio, "drop_rate": drop_rate, "attn_drop_rate": attn_drop_rate,
            "dropout_path_rate": dropout_path_rate, "use_checkpoint": use_checkpoint,
            "norm_name": norm_name, "lr": lr, "weight_decay": weight_decay,
            "warmup_epochs": warmup_epochs, "use_ce_alongside_dice": use_ce_alongside_dice,
            "ce_weight": ce_weight, "ignore_index": ignore_index,
            "include_bg_in_dice": include_bg_in_dice})
        self.model = SwinUNETR_Published(
            num_classes, img_size=img_size, in_channels=in_channels, feature_size=feature_size,
            depths=depths, num_heads=num_heads, mlp_ratio=mlp_ratio, drop_rate=drop_rate,
            attn_drop_rate=attn_drop_rate, dropout_path_rate=dropout_path_rate,
            use_checkpoint=use_checkpoint, norm_name=norm_name)
        self._total_train_iters = None
        self._iters_done = 0

    def forward(self, x):
        x = _pick_first_if_seq(x)
        if x.ndim == 4:
            x = x.unsqueeze(1)
        x_pad, orig = _pad_to_mult16_3d(x, multiple=32)
        y_pad = self.model(x_pad)
        return _center_crop_3d(y_pad, orig)

    def _loss(self, logits, labels):
        if labels.ndim == 5 and labels.shape[1] == 1:
            labels = labels[:, 0]
        if not self.hparams.use_ce_alongside_dice:
            raise NotImplementedError("dice-only loss is off on the registry path (config.py:383)")
        ign = self.hparams.ignore_index
        return _SwinLoss.apply(logits, labels, int(logits.shape[1]),
                               int(ign) if ign is not None else -1000,
                               bool(self.hparams.include_bg_in_dice), float(self.hparams.ce_weight))

    def on_train_batch_start(self, batch, batch_idx):
        """linear warm-up then cosine decay of the learning rate (models.py:941-951)."""
        tr = getattr(self, "trainer", None)
        nb = int(getattr(tr, "num_training_batches", 0) or 1) if tr is not None else 1
        warmup_iters = int(self.hparams.warmup_epochs * nb)
        t, T = self._iters_done, max(1, self._total_train_iters or 1)
        if t < warmup_iters:
            lr = self.hparams.lr * float(t + 1) / max(1, warmup_iters)
        else:
            prog = (t - warmup_iters) / max(1, T - warmup_iters)
            lr = 0.5 * self.hparams.lr * (1.0 + math.cos(math.pi * prog))
        opt = self.optimizers() if hasattr(self, "optimizers") and tr is not None else None
        if opt:
            for pg in opt.param_groups:
                pg["lr"] = lr
        return lr

    def on_train_batch_end(self, outputs, batch, batch_idx):
        self._iters_done += 1

    def _step(self, batch, stage):
        imgs, lbls = batch if isinstance(batch, (list, tuple)) else (batch["image"], batch["label"])
        logits = self(imgs)
        tgt = _canonicalize_targets_3d(lbls).to(logits.device)
        loss = self._loss(logits, tgt)
        met = per_class_metrics_3d(logits, tgt, self.hparams.num_classes,
                                   ignore_index=self.hparams.ignore_index)
        self.log(f"{stage}_loss", loss, on_epoch=True, prog_bar=True, sync_dist=True)
        self.log(f"{stage}_macro_dice", met[3], on_epoch=True, prog_bar=True, sync_dist=True)
        self.log(f"{stage}_micro_dice", met[6], on_epoch=True, prog_bar=False, sync_dist=True)
        return loss

    def training_step(self, batch, _):
        return self._step(batch, "train")

    def validation_step(self, batch, _):
        return self._step(batch, "val")

    def test_step(self, batch, _):
        return self._step(batch, "test")

    def configure_optimizers(self):
        return torch.optim.AdamW(self.parameters(), lr=self.hparams.lr,
                                 weight_decay=self.hparams.weight_decay, betas=(0.9, 0.999))
