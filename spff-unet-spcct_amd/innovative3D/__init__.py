"""innovative3D -- MI355X-native drop-in for the reference package of the same
name (NF-91/spff-unet-spcct).  The SPFF-UNet forward / loss / backward run in
libspff_hip.so (hand-written HIP for gfx950, see include/spff.h); this package
keeps the reference's Python surface: config.VARIANTS, the LitSPCT_* modules,
helpers.ce_plus_macro_dice_loss / per_class_metrics_3d, unified_loss and
unified_optimizer.  (The reference ships a misnamed ``_init_.py``, so it
imports as a namespace package; this one is a regular package.)
"""
__version__ = "0.1.0"
