"""CPU ORACLE for the SwinUNETR variant -- TEST INFRASTRUCTURE ONLY.

A from-scratch functional restatement, in plain PyTorch-CPU, of the
reference's "SwinUNETR" registry entry (config.py:366-386):
LitSwinUNETR_Published (models.py:880-982) around SwinUNETR_Published
(models.py:858-878), which builds ``monai.networks.nets.SwinUNETR``.  Backward
is PyTorch autograd over this graph.  Imported ONLY by ``tests/`` (and the
bench's CPU-baseline leg) as the checker -- never by the product path.

PARITY UNPINNED.  MONAI is a third-party dependency absent from
/root/reference and from this image (``monai==1.5.2``, requirements.txt:40);
the reference ships no test, fixture or golden output for this model, and
nothing from MONAI can be run here.  This file restates MONAI 1.5.2's
published SwinUNETR semantics as the registry instantiates them:

* ``build_class`` passes only the kwargs LitSwinUNETR_Published accepts
  (config.py:159-182); ``window_size=(2,2,2)`` is NOT among them
  (models.py:882-889), so MONAI's default ``window_size=7`` applies.
  feature_size 12, depths (1,1,1,1), heads (1,2,4,8), mlp_ratio 2, qkv_bias,
  norm_name "instance", normalize=True, patch_size 2, downsample "merging"
  (MONAI's legacy ``PatchMerging``), use_v2=False, dropout 0, and
  ``img_size`` dropped (MONAI 1.5 has no such argument; models.py:870-874).
* depth 1 per stage => every Swin block is the unshifted one (shift only for
  odd block indices), so no attention mask.  Tokens padded up to a window
  multiple AFTER norm1 are zeros that DO take part in attention as keys /
  values (their k, v are the qkv bias); their outputs are cropped.
* relative position bias: table[(2w-1)^3, heads] indexed by the w^3 window's
  pairwise index, sliced ``[:n, :n]`` when a stage's window shrinks to the
  volume (x_size <= w).
* PatchMerging (legacy): cat of the 8 stride-2 slices in MONAI's order
  (0,0,0),(1,0,0),(0,1,0),(0,0,1),(1,0,1),(0,1,0),(0,0,1),(1,1,1) -- the
  duplicated (0,1,0)/(0,0,1) slices are MONAI's kept-for-compatibility quirk --
  then LayerNorm(8C) and Linear(8C -> 2C, no bias).
* proj_out(normalize=True): affine-free layer norm over channels of each
  hidden state.
* UnetrBasicBlock(res_block=True) = UnetResBlock: conv3 -> IN -> lrelu ->
  conv3 -> IN, plus (1x1 conv -> IN) shortcut when cin != cout, add, lrelu;
  InstanceNorm3d without affine, LeakyReLU 0.01, convs without bias.
  UnetrUpBlock: ConvTranspose3d(k=2, s=2, no bias), cat [up, skip],
  UnetResBlock.  UnetOutBlock: 1x1 conv with bias.
* Lit loss (models.py:910-928): (1-w) * soft-Dice loss + w * CE(ignore 255),
  w = ce_weight = 0.5; soft Dice over classes >= 1 (include_bg_in_dice False),
  probabilities masked by the valid voxels, one-hot of the labels with the
  ignored voxels mapped to class 0, dice = mean over (b, c) of
  2 sum(p g) / (sum p + sum g + 1e-6).
"""
from __future__ import annotations

import itertools
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

__all__ = ["SwinCfg", "param_shapes", "buffer_shapes", "rel_index", "forward", "lit_loss",
           "fwd_bwd", "params_from_state", "STAGE_MERGE_ORDER"]

# PatchMerging (legacy) slice order: (d, h, w) offsets of x0..x7
STAGE_MERGE_ORDER = ((0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (0, 1, 0), (0, 0, 1),
                     (1, 1, 1))


@dataclass
class SwinCfg:
    num_classes: int = 13
    in_ch: int = 1
    feature_size: int = 12
    depths: Tuple[int, ...] = (1, 1, 1, 1)
    num_heads: Tuple[int, ...] = (1, 2, 4, 8)
    window: int = 7
    mlp_ratio: float = 2.0
    ce_weight: float = 0.5
    include_bg_in_dice: bool = False
    ignore_index: int = 255


def _resblock_shapes(out, name, ci, co):
    out.append((f"{name}.conv1.conv.weight", (co, ci, 3, 3, 3)))
    out.append((f"{name}.conv2.conv.weight", (co, co, 3, 3, 3)))
    if ci != co:
        out.append((f"{name}.conv3.conv.weight", (co, ci, 1, 1, 1)))


def param_shapes(cfg: SwinCfg, prefix: str = "") -> "OrderedDict[str, Tuple[int, ...]]":
    """Parameters in MONAI SwinUNETR registration order (swinViT, encoder1..4,
    encoder10, decoder5..1, out)."""
    if any(d != 1 for d in cfg.depths):
        raise NotImplementedError("depths (1,1,1,1) only (the registry's; config.py:374)")
    f, p, w = cfg.feature_size, prefix, cfg.window
    out: List[Tuple[str, Tuple[int, ...]]] = []
    out.append((p + "swinViT.patch_embed.proj.weight", (f, cfg.in_ch, 2, 2, 2)))
    out.append((p + "swinViT.patch_embed.proj.bias", (f,)))
    for s in range(4):
        C, nh = f << s, cfg.num_heads[s]
        hid = int(C * cfg.mlp_ratio)
        b = f"{p}swinViT.layers{s + 1}.0.blocks.0."
        out += [(b + "norm1.weight", (C,)), (b + "norm1.bias", (C,)),
                (b + "attn.relative_position_bias_table", ((2 * w - 1) ** 3, nh)),
                (b + "attn.qkv.weight", (3 * C, C)), (b + "attn.qkv.bias", (3 * C,)),
                (b + "attn.proj.weight", (C, C)), (b + "attn.proj.bias", (C,)),
                (b + "norm2.weight", (C,)), (b + "norm2.bias", (C,)),
                (b + "mlp.linear1.weight", (hid, C)), (b + "mlp.linear1.bias", (hid,)),
                (b + "mlp.linear2.weight", (C, hid)), (b + "mlp.linear2.bias", (C,))]
        d = f"{p}swinViT.layers{s + 1}.0.downsample."
        out += [(d + "reduction.weight", (2 * C, 8 * C)), (d + "norm.weight", (8 * C,)),
                (d + "norm.bias", (8 * C,))]
    _resblock_shapes(out, p + "encoder1.layer", cfg.in_ch, f)
    _resblock_shapes(out, p + "encoder2.layer", f, f)
    _resblock_shapes(out, p + "encoder3.layer", 2 * f, 2 * f)
    _resblock_shapes(out, p + "encoder4.layer", 4 * f, 4 * f)
    _resblock_shapes(out, p + "encoder10.layer", 16 * f, 16 * f)
    for name, ci, co in (("decoder5", 16 * f, 8 * f), ("decoder4", 8 * f, 4 * f),
                         ("decoder3", 4 * f, 2 * f), ("decoder2", 2 * f, f), ("decoder1", f, f)):
        out.append((f"{p}{name}.transp_conv.conv.weight", (ci, co, 2, 2, 2)))
        _resblock_shapes(out, f"{p}{name}.conv_block", 2 * co, co)
    out.append((p + "out.conv.conv.weight", (cfg.num_classes, f, 1, 1, 1)))
    out.append((p + "out.conv.conv.bias", (cfg.num_classes,)))
    return OrderedDict(out)


def rel_index(w: int) -> torch.Tensor:
    """[w^3, w^3] int64 pairwise index into the (2w-1)^3 bias table (the
    ``relative_position_index`` buffer)."""
    c = torch.stack(torch.meshgrid(torch.arange(w), torch.arange(w), torch.arange(w),
                                   indexing="ij")).flatten(1)          # [3, n]
    r = (c[:, :, None] - c[:, None, :]).permute(1, 2, 0) + (w - 1)   # [n, n, 3]
    return r[..., 0] * (2 * w - 1) ** 2 + r[..., 1] * (2 * w - 1) + r[..., 2]


def buffer_shapes(cfg: SwinCfg, prefix: str = "") -> "OrderedDict[str, Tuple[int, ...]]":
    n = cfg.window ** 3
    return OrderedDict((f"{prefix}swinViT.layers{s + 1}.0.blocks.0.attn.relative_position_index",
                        (n, n)) for s in range(4))


def _ln_c(x, weight=None, bias=None):
    """layer norm over the channel dim of [B, C, D, H, W] (eps 1e-5)."""
    y = F.layer_norm(x.permute(0, 2, 3, 4, 1), (x.shape[1],), weight, bias, eps=1e-5)
    return y.permute(0, 4, 1, 2, 3).contiguous()


def _window_attention(P, pre, x, nh, w, ridx):
    """x: [B, D, H, W, C] (already norm1'd).  One unshifted Swin attention."""
    B, D, H, W, C = x.shape
    ws = [min(w, s) for s in (D, H, W)]
    pd, ph, pw = [(k - s % k) % k for k, s in zip(ws, (D, H, W))]
    xp = F.pad(x, (0, 0, 0, pw, 0, ph, 0, pd))
    Dp, Hp, Wp = D + pd, H + ph, W + pw
    n = ws[0] * ws[1] * ws[2]
    win = xp.view(B, Dp // ws[0], ws[0], Hp // ws[1], ws[1], Wp // ws[2], ws[2], C)
    win = win.permute(0, 1, 3, 5, 2, 4, 6, 7).reshape(-1, n, C)
    qkv = F.linear(win, P[pre + "qkv.weight"], P[pre + "qkv.bias"])
    qkv = qkv.reshape(-1, n, 3, nh, C // nh).permute(2, 0, 3, 1, 4)
    q, k, v = qkv[0] * (C // nh) ** -0.5, qkv[1], qkv[2]
    a = q @ k.transpose(-2, -1)
    tab = P[pre + "relative_position_bias_table"]
    bias = tab[ridx[:n, :n].reshape(-1)].reshape(n, n, -1).permute(2, 0, 1)
    a = torch.softmax(a + bias.unsqueeze(0), dim=-1)
    o = (a @ v).transpose(1, 2).reshape(-1, n, C)
    o = F.linear(o, P[pre + "proj.weight"], P[pre + "proj.bias"])
    o = o.view(B, Dp // ws[0], Hp // ws[1], Wp // ws[2], ws[0], ws[1], ws[2], C)
    o = o.permute(0, 1, 4, 2, 5, 3, 6, 7).reshape(B, Dp, Hp, Wp, C)
    return o[:, :D, :H, :W, :]


def _swin_block(P, pre, x, nh, w, ridx):
    """x: [B, D, H, W, C] -> same (SwinTransformerBlock, no shift)."""
    C = x.shape[-1]
    h = F.layer_norm(x, (C,), P[pre + "norm1.weight"], P[pre + "norm1.bias"], eps=1e-5)
    x = x + _window_attention(P, pre + "attn.", h, nh, w, ridx)
    h = F.layer_norm(x, (C,), P[pre + "norm2.weight"], P[pre + "norm2.bias"], eps=1e-5)
    h = F.gelu(F.linear(h, P[pre + "mlp.linear1.weight"], P[pre + "mlp.linear1.bias"]))
    return x + F.linear(h, P[pre + "mlp.linear2.weight"], P[pre + "mlp.linear2.bias"])


def _merge(P, pre, x):
    """legacy PatchMerging on [B, D, H, W, C] -> [B, D/2, H/2, W/2, 2C]."""
    B, D, H, W, C = x.shape
    if D % 2 or H % 2 or W % 2:
        x = F.pad(x, (0, 0, 0, W % 2, 0, H % 2, 0, D % 2))
    x = torch.cat([x[:, a::2, b::2, c::2, :] for a, b, c in STAGE_MERGE_ORDER], -1)
    x = F.layer_norm(x, (8 * C,), P[pre + "norm.weight"], P[pre + "norm.bias"], eps=1e-5)
    return F.linear(x, P[pre + "reduction.weight"])


def _in(x):
    return F.instance_norm(x, eps=1e-5)


# Optional LeakyReLU sign patterns {"<block prefix>act1" / "act2": bool [B,C,D,H,W]}:
# tests set this to the engine's own signs so a fp32 knife-edge input (|x| ~ 0)
# takes the same slope in both (kink-consistent gradients); None = plain lrelu.
ACT_MASKS: Optional[Dict[str, torch.Tensor]] = None


def _lrelu(name, t):
    if ACT_MASKS is None:
        return F.leaky_relu(t, 0.01)
    return torch.where(ACT_MASKS[name], t, 0.01 * t)


def _resblock(P, pre, x):
    y = _lrelu(pre + "act1", _in(F.conv3d(x, P[pre + "conv1.conv.weight"], padding=1)))
    y = _in(F.conv3d(y, P[pre + "conv2.conv.weight"], padding=1))
    r = x
    if pre + "conv3.conv.weight" in P:
        r = _in(F.conv3d(x, P[pre + "conv3.conv.weight"]))
    return _lrelu(pre + "act2", y + r)


def _upblock(P, pre, x, skip):
    u = F.conv_transpose3d(x, P[pre + "transp_conv.conv.weight"], stride=2)
    return _resblock(P, pre + "conv_block.", torch.cat([u, skip], 1))


def forward(P: Dict[str, torch.Tensor], x: torch.Tensor, cfg: SwinCfg, prefix: str = "",
            taps: Optional[dict] = None) -> torch.Tensor:
    """MONAI SwinUNETR.forward on [B, Cin, D, H, W] (D, H, W multiples of 32)."""
    p = prefix
    if any(s % 32 for s in x.shape[2:]):
        raise ValueError("SwinUNETR needs D, H, W divisible by 2**5 = 32")
    w = cfg.window
    ridx = rel_index(w)
    x0 = F.conv3d(x, P[p + "swinViT.patch_embed.proj.weight"],
                  P[p + "swinViT.patch_embed.proj.bias"], stride=2)
    hs = [_ln_c(x0)]
    t = x0
    for s in range(4):
        pre = f"{p}swinViT.layers{s + 1}.0."
        tl = t.permute(0, 2, 3, 4, 1)
        tl = _swin_block(P, pre + "blocks.0.", tl, cfg.num_heads[s], w, ridx)
        tl = _merge(P, pre + "downsample.", tl)
        t = tl.permute(0, 4, 1, 2, 3)
        hs.append(_ln_c(t))
    enc0 = _resblock(P, p + "encoder1.layer.", x)
    enc1 = _resblock(P, p + "encoder2.layer.", hs[0])
    enc2 = _resblock(P, p + "encoder3.layer.", hs[1])
    enc3 = _resblock(P, p + "encoder4.layer.", hs[2])
    dec4 = _resblock(P, p + "encoder10.layer.", hs[4])
    dec3 = _upblock(P, p + "decoder5.", dec4, hs[3])
    dec2 = _upblock(P, p + "decoder4.", dec3, enc3)
    dec1 = _upblock(P, p + "decoder3.", dec2, enc2)
    dec0 = _upblock(P, p + "decoder2.", dec1, enc1)
    out = _upblock(P, p + "decoder1.", dec0, enc0)
    if taps is not None:
        taps.update(x0=x0, hs=hs, enc0=enc0, enc1=enc1, enc2=enc2, enc3=enc3, dec4=dec4,
                    dec3=dec3, dec2=dec2, dec1=dec1, dec0=dec0, out=out)
    return F.conv3d(out, P[p + "out.conv.conv.weight"], P[p + "out.conv.conv.bias"])


def lit_loss(logits: torch.Tensor, labels: torch.Tensor, cfg: SwinCfg) -> torch.Tensor:
    """LitSwinUNETR_Published._loss (models.py:910-928)."""
    if labels.ndim == 5 and labels.shape[1] == 1:
        labels = labels[:, 0]
    C = logits.shape[1]
    probs = torch.softmax(logits, dim=1)
    ign = cfg.ignore_index
    mask = (labels != ign).unsqueeze(1).to(logits.dtype)
    lab = torch.where(labels == ign, torch.zeros_like(labels), labels)
    probs = probs * mask
    onehot = F.one_hot(lab.clamp_min(0), num_classes=C).permute(0, 4, 1, 2, 3).to(logits.dtype)
    sc = 0 if cfg.include_bg_in_dice else 1
    pp, g = probs[:, sc:], onehot[:, sc:]
    inter = (pp * g).sum(dim=(2, 3, 4))
    den = pp.sum(dim=(2, 3, 4)) + g.sum(dim=(2, 3, 4)) + 1e-6
    dice = 1.0 - (2 * inter / den).mean()
    ce = F.cross_entropy(logits, labels, ignore_index=ign)
    w = float(cfg.ce_weight)
    return (1.0 - w) * dice + w * ce


def params_from_state(state, requires_grad=True, dtype=torch.float32, prefix=""):
    P = {}
    for k, v in state.items():
        if not k.startswith(prefix) or k.endswith("relative_position_index"):
            continue
        t = torch.as_tensor(v).to(dtype).clone()
        t.requires_grad_(requires_grad)
        P[k[len(prefix):]] = t
    return P


def fwd_bwd(P, x, labels, cfg: SwinCfg):
    """forward + Lit loss + backward; returns (logits, loss)."""
    for t in P.values():
        t.grad = None
    logits = forward(P, x.to(next(iter(P.values())).dtype), cfg)
    loss = lit_loss(logits, labels, cfg)
    loss.backward()
    return logits.detach(), loss.detach()
