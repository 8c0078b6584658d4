"""Registry and constants (mirror of innovative3D/config.py).

Keeps the reference's registry contract -- ``VARIANTS`` is a list of
``(name, factory, DataModuleCls, ckpt_dir)`` tuples built through
``build_class`` (config.py:159-182, 271-280) -- for the SPCT/SPFF family the
engine implements.  Differences, all deliberate:

* no import-time side effects: the reference mkdirs a hard-coded /home path
  and CHECKPOINT_DIR/LOG_DIR at import (config.py:19, 258-259); here
  directories are created by whoever writes to them (train.py);
* ``INNOVATIVE3D_VARIANT`` actually selects: ``selected_variants()``;
* of the non-SPCT baselines "3DUNet" (BASELINE config 3, SURVEY §8(f) rank 2:
  Cicek3DUNet + depth adapter) and "SwinUNETR" (BASELINE config 5, §8(f) rank 3)
  are registered, both on the engine; UNETR, R2UNet3D and ResUNet++ are outside
  the SPFF hot path;
* the DICOM data module (``MultiDicomDataModule3D``) is the device-resident
  one of innovative3D/datasets.py (resize, ROI rasterisation and TrainGridAug as
  HIP kernels); DICOM files are decoded by pydicom when installed, else by the native
  reader of innovative3D/dicom.py (uncompressed transfer syntaxes).
"""
from __future__ import annotations

import inspect
import os
from importlib import import_module
from pathlib import Path

os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")

IMAGE_HEIGHT, IMAGE_WIDTH = 512, 512
NUM_FRAMES = 5
NUM_CLASSES = 13
FINAL_EPOCHS = 200
BEST_LR = 1e-4
IGNORE_INDEX = 255
BATCH_SIZE = 1
NUM_WORKERS = 16
num_workers = NUM_WORKERS
grid_size = 10
SEEDS = [42, 123, 999]

global_label_names = {
    0: "BG", 1: "HA800", 2: "HA400", 3: "HA200", 4: "HA100", 5: "Lung", 6: "Liver", 7: "Adipose",
    8: "Water", 9: "I15", 10: "I10", 11: "I5", 12: "HA50",
}

LOSS_NAME = "ce_plus_macro_dice"

BASE_DIR = Path(os.getenv("SPFF_BASE_DIR", str(Path.home() / "spff_runs")))
CHECKPOINT_DIR = Path(os.getenv("CHECKPOINT_DIR", str(BASE_DIR / "checkpoints"))).resolve()
LOG_DIR = Path(os.getenv("LOG_DIR", str(BASE_DIR / "runs"))).resolve()
CKPT_DIR = CHECKPOINT_DIR


def MultiDicomDataModule3D(*args, **kwargs):
    """datasets.py:280-338 on the device (innovative3D/datasets.py)."""
    from .datasets import MultiDicomDataModule3D as _DM
    return _DM(*args, **kwargs)


MultiDicomDataModule2D = MultiDicomDataModule3D


def build_from_models(func_name: str, **fixed_kwargs):
    def _factory():
        mod = import_module("innovative3D.models")
        fn = getattr(mod, func_name, None)
        if fn is None:
            raise ImportError(f"[config] {func_name} not found in innovative3D.models")
        return fn(**fixed_kwargs)
    return _factory


def build_class(class_name: str, **ctor_kwargs):
    """Factory that filters kwargs by the constructor signature (config.py:159-182).
    Call-time keyword overrides (e.g. ``in_channels=5`` for the north-star
    5-bin-as-channels layout) are merged over the registered ones."""
    def _factory(**overrides):
        ctor = {**ctor_kwargs, **overrides}
        mod = import_module("innovative3D.models")
        cls = getattr(mod, class_name, None)
        if cls is None:
            raise ImportError(f"[config] {class_name} not found in innovative3D.models")
        try:
            sig = inspect.signature(cls.__init__)
            if any(p.kind == inspect.Parameter.VAR_KEYWORD for p in sig.parameters.values()):
                filtered = dict(ctor)
            else:
                allowed = {n for n in sig.parameters if n != "self"}
                filtered = {k: v for k, v in ctor.items() if k in allowed}
        except (TypeError, ValueError):
            filtered = dict(ctor)
        return cls(**filtered)
    return _factory


VARIANTS = []


def _add_variant(name, builder_or_class, dm_cls, ckpt_dir):
    VARIANTS.append((name, builder_or_class, dm_cls, Path(ckpt_dir)))


_SPCT_COMMON = dict(num_classes=NUM_CLASSES, lr=BEST_LR, base=32, ksd=3, use_se=True,
                    use_specse=True, use_spatial=False, use_skip_gate=False)

_add_variant("SPFF-UNet", build_class("LitSPCT_EFiLM_FourierGate", **_SPCT_COMMON),
             MultiDicomDataModule3D, CHECKPOINT_DIR / "SPFF-UNet")
_add_variant("E_SP_UNet", build_class("LitSPCT_EnergyFiLM", **_SPCT_COMMON),
             MultiDicomDataModule3D, CHECKPOINT_DIR / "E_SP_UNet")
_add_variant("FG_SP_UNet", build_class("LitSPCT_FourierGate", **_SPCT_COMMON),
             MultiDicomDataModule3D, CHECKPOINT_DIR / "FG_SP_UNet")
_add_variant("SP_UNet", build_class("LitSPCT_SEspec", num_classes=NUM_CLASSES, lr=BEST_LR),
             MultiDicomDataModule3D, CHECKPOINT_DIR / "SP_UNet")
_plaincore_kwargs = {**_SPCT_COMMON, "use_se": False, "use_specse": False, "use_spatial": False,
                     "use_skip_gate": False}
_add_variant("PlainCore_UNet", build_class("LitSPCT_ControlUNet", **_plaincore_kwargs),
             MultiDicomDataModule3D, CHECKPOINT_DIR / "PlainCore_UNet")



def make_cicek_depth_adapter_sgd_wce():
    """config.py:283-303: Cicek 3D U-Net + depth adapter, SGD, weighted CE."""
    from innovative3D.models import LitCicek3DUNet_DepthAdapter_Published
    return LitCicek3DUNet_DepthAdapter_Published(
        num_classes=NUM_CLASSES,
        lr=1e-2, momentum=0.99, nesterov=False, weight_decay=0.0,   # SGD like the paper
        ignore_index=255, class_weights=None, voxel_weight_key=None,  # weighted softmax CE
        ce_weight=1.0, dice_weight=0.0,
        use_bn=True, target_depth=16, include_bg_in_dice=False,
    )


_add_variant("3DUNet", make_cicek_depth_adapter_sgd_wce, MultiDicomDataModule3D,
             CHECKPOINT_DIR / "3DUNet")

# SwinUNETR (config.py:366-386; BASELINE config 5).  build_class drops the kwargs
# LitSwinUNETR_Published does not take (window_size), exactly like the reference.
_add_variant("SwinUNETR",
             build_class("LitSwinUNETR_Published", num_classes=NUM_CLASSES, img_size=(64, 64, 64),
                         in_channels=1, feature_size=12, depths=(1, 1, 1, 1),
                         num_heads=(1, 2, 4, 8), window_size=(2, 2, 2), mlp_ratio=2.0,
                         drop_rate=0.0, attn_drop_rate=0.0, dropout_path_rate=0.0,
                         norm_name="instance", use_checkpoint=True, lr=8e-4, weight_decay=1e-2,
                         warmup_epochs=5, use_ce_alongside_dice=True, ce_weight=0.5,
                         ignore_index=IGNORE_INDEX, include_bg_in_dice=False),
             MultiDicomDataModule3D, CHECKPOINT_DIR / "SwinUNETR")

VARIANT_NAMES = [v[0] for v in VARIANTS]
SELECTED_VARIANT = os.getenv("INNOVATIVE3D_VARIANT")


def selected_variants():
    """Variants to run: INNOVATIVE3D_VARIANT (comma list) if set, else all."""
    sel = os.getenv("INNOVATIVE3D_VARIANT", SELECTED_VARIANT or "")
    if not sel:
        return list(VARIANTS)
    names = [s.strip() for s in sel.split(",") if s.strip()]
    unknown = [n for n in names if n not in VARIANT_NAMES]
    if unknown:
        raise KeyError(f"unknown variant(s) {unknown}; known: {VARIANT_NAMES}")
    return [v for v in VARIANTS if v[0] in names]


def variant(name: str):
    for v in VARIANTS:
        if v[0] == name:
            return v
    raise KeyError(f"unknown variant {name}; known: {VARIANT_NAMES}")
