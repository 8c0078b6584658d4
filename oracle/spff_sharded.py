"""TEST INFRASTRUCTURE -- depth-sharded restatement of the SPFF path (CPU).

Only tests/ may import this.  It restates the reference forward (models.py
647-701, 1448-1555) for a volume split along D across the ranks of a
torch.distributed group -- BASELINE config 4 / SURVEY.md §8(e) "depth
sharding" -- using DIFFERENTIABLE collectives, so one local backward per rank
followed by the flat gradient all-reduce reproduces the unsharded gradients.
It is the algorithmic contract the engine's sharded plans follow:

  * 3x3x3 conv: one D-slice halo per side from the neighbouring ranks, zeros at
    the global ends (here: an all-gather of the boundary slices);
  * InstanceNorm3d: per-(b,c) sum and sum of squared deviations all-reduced
    (two-pass, as the engine);
  * FourierGate: s1[b, d] is per-slice (mean over c, h, w), so it is all-gathered
    to the full D, the rfft/mask/irfft is evaluated replicated and each rank
    keeps its own slice of the gate;
  * SpectralSE: per slice, rank-local;  channel SE: pool all-reduced;
  * EnergyFiLM: the positional encoding at the GLOBAL depth indices;
  * pool / ConvTranspose / 1x1 head / concat: rank-local;
  * loss: CE summed locally over the GLOBAL valid count (all-reduced), the
    hard-Dice term from the all-reduced confusion.

Batch B is arbitrary here (the engine's sharded plans take B = 1)."""
from __future__ import annotations

from typing import Dict, Tuple

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch.distributed.nn.functional import all_gather, all_reduce

from oracle import spff_oracle as O


class Shard:
    """Rank r of `world` owns global indices [off, off + D_loc) along ``axis`` (2 = D,
    3 = H) of a volume whose extent along that axis is D."""

    def __init__(self, D: int, rank: int, world: int, axis: int = 2):
        if D % world:
            raise ValueError(f"extent {D} not divisible by world={world}")
        if axis not in (2, 3):
            raise ValueError("axis must be 2 (depth) or 3 (height)")
        self.D, self.rank, self.world, self.axis = D, rank, world, axis
        self.D_loc = D // world
        self.off = rank * self.D_loc
        if axis == 3 and self.D_loc % 8:
            raise ValueError("height shards must hold a multiple of 8 rows (three (1,2,2) pools)")

    def n_glob(self, x: torch.Tensor) -> int:
        """voxels per (b, c) of the global volume at x's level"""
        n = x.shape[2] * x.shape[3] * x.shape[4]
        return n * self.world


def halo_pad(x: torch.Tensor, sh: Shard, k: int) -> torch.Tensor:
    """[B, C, D_loc, H, W] -> [B, C, D_loc + 2k, H, W] with k neighbour slices per
    side (zeros beyond the global ends); along H for a height shard."""
    if k == 0:
        return x
    ax = sh.axis
    firsts = all_gather(x.narrow(ax, 0, k).contiguous())
    lasts = all_gather(x.narrow(ax, x.shape[ax] - k, k).contiguous())
    # Every gathered output stays in the graph on every rank (x 0 at the global
    # ends): autograd skips a node none of whose outputs is used, and a
    # collective's backward must run on all ranks in the same order.
    left = lasts[sh.rank - 1] if sh.rank > 0 else lasts[0] * 0
    right = firsts[sh.rank + 1] if sh.rank + 1 < sh.world else firsts[-1] * 0
    return torch.cat([left, x, right], dim=ax)


def instance_norm(y, w, b, sh: Shard, eps=1e-5):
    n = sh.n_glob(y)
    mean = all_reduce(y.sum(dim=(2, 3, 4), keepdim=True)) / n
    var = all_reduce(((y - mean) ** 2).sum(dim=(2, 3, 4), keepdim=True)) / n
    return (y - mean) / torch.sqrt(var + eps) * w[None, :, None, None, None] + b[None, :, None, None, None]


def conv_in_lrelu(P, pre, x, ksd, sh: Shard):
    if sh.axis == 2:
        xp = halo_pad(x, sh, ksd // 2)
        y = F.conv3d(xp, P[pre + ".0.weight"], None, padding=(0, 1, 1))
    else:
        xp = halo_pad(x, sh, 1)
        y = F.conv3d(xp, P[pre + ".0.weight"], None, padding=(ksd // 2, 0, 1))
    y = instance_norm(y, P[pre + ".1.weight"], P[pre + ".1.bias"], sh)
    return F.leaky_relu(y, 0.01)


def energy_film(P, pre, x, sh: Shard):
    C = x.shape[1]
    if sh.axis == 3:
        return O.energy_film(P, pre, x)
    g, b = O.energy_film_gb(P, pre, C, sh.D)
    g, b = g[..., sh.off:sh.off + sh.D_loc], b[..., sh.off:sh.off + sh.D_loc]
    return x * (1 + g[..., None, None]) + b[..., None, None]


def fourier_gate(P, pre, x, sh: Shard, learn_phase: bool = False):
    if sh.axis == 3:   # s1 = mean over (c, h, w): partial sums over the local rows
        B, C, Fd, H, W = x.shape
        s_full = all_reduce(x.sum(dim=(1, 3, 4))) / (C * H * sh.world * W)
        Sf = O.host_rfft(s_full, dim=1)
        M = (P[pre + ".freq_mask"] * P[pre + ".mag_scale"]).reshape(1, -1)
        w = O.host_irfft(Sf * (M + 1j * 0.01) if learn_phase else Sf * M, n=Fd, dim=1)
        return x * torch.sigmoid(w)[:, None, :, None, None]
    s = x.mean(dim=(1, 3, 4))                              # [B, D_loc]
    s_full = torch.cat(all_gather(s.contiguous()), dim=1)   # [B, D]
    Sf = O.host_rfft(s_full, dim=1)
    M = (P[pre + ".freq_mask"] * P[pre + ".mag_scale"]).reshape(1, -1)
    Sf = Sf * (M + 1j * 0.01) if learn_phase else Sf * M
    w = O.host_irfft(Sf, n=sh.D, dim=1)[:, sh.off:sh.off + sh.D_loc]
    return x * torch.sigmoid(w)[:, None, :, None, None]


def spectral_se(x, sh: Shard):
    """models.py:611-614: per-slice mean over (c, h, w) -- rank-local for a depth
    shard, all-reduced partial sums for a height shard"""
    if sh.axis == 2:
        return O.spectral_se(x)
    B, C, Fd, H, W = x.shape
    m = all_reduce(x.sum(dim=(1, 3, 4), keepdim=True)) / (C * H * sh.world * W)
    return x * torch.sigmoid(m)


def se_channel(P, pre, x, sh: Shard):
    n = sh.n_glob(x)
    p = (all_reduce(x.sum(dim=(2, 3, 4), keepdim=True)) / n)
    h = F.relu(F.conv3d(p, P[pre + ".fc.0.weight"], P[pre + ".fc.0.bias"]))
    e = torch.sigmoid(F.conv3d(h, P[pre + ".fc.2.weight"], P[pre + ".fc.2.bias"]))
    return x * e


def novel_block(P, pre, x, cfg, sh: Shard):
    a, b = ("pre", "body") if cfg.novel else ("b1", "b2")
    x = conv_in_lrelu(P, f"{pre}.{a}", x, cfg.ksd, sh)
    x = conv_in_lrelu(P, f"{pre}.{b}", x, cfg.ksd, sh)
    if cfg.novel and cfg.efilm:
        x = energy_film(P, pre + ".efilm", x, sh)
    if cfg.novel and cfg.fgate:
        x = fourier_gate(P, pre + ".fgate", x, sh, cfg.learn_phase)
    return x


def _post(P, x, stage, cfg, sh: Shard):
    if cfg.specse:
        x = spectral_se(x, sh)
    if cfg.se:
        x = se_channel(P, f"se.{stage}", x, sh)
    return x


def forward(P: Dict[str, torch.Tensor], x_loc: torch.Tensor, cfg, sh: Shard) -> torch.Tensor:
    """Local logits [B, K, D_loc, H, W] (height shard: [B, K, D, H_loc, W]) of
    UNet3D_SpectralCore.forward."""
    pool = lambda t: F.max_pool3d(t, (1, 2, 2))  # noqa: E731
    up = lambda t, n: F.conv_transpose3d(t, P[n + ".weight"], P[n + ".bias"], stride=(1, 2, 2))  # noqa: E731
    e1 = _post(P, novel_block(P, "enc1", x_loc, cfg, sh), 0, cfg, sh)
    e2 = _post(P, novel_block(P, "enc2", pool(e1), cfg, sh), 1, cfg, sh)
    e3 = _post(P, novel_block(P, "enc3", pool(e2), cfg, sh), 2, cfg, sh)
    b = _post(P, novel_block(P, "bott", pool(e3), cfg, sh), 3, cfg, sh)
    d3 = novel_block(P, "dec3", O._cat(up(b, "up3"), e3), cfg, sh)
    d2 = novel_block(P, "dec2", O._cat(up(d3, "up2"), e2), cfg, sh)
    d1 = novel_block(P, "dec1", O._cat(up(d2, "up1"), e1), cfg, sh)
    return F.conv3d(d1, P["out.weight"], P["out.bias"])


def fwd_bwd(P, x_loc, y_loc, cfg, sh: Shard, ignore_index=255) -> Tuple[float, float, float]:
    """Local forward + the global ce_plus_macro_dice loss + local backward, then
    the flat gradient all-reduce.  Returns the global (loss, ce, dice_loss)."""
    logits = forward(P, x_loc, cfg, sh)
    K = logits.shape[1]
    n = (y_loc != ignore_index).sum().to(torch.float64).reshape(1)
    dist.all_reduce(n)
    ce_loc = F.cross_entropy(logits, y_loc, ignore_index=ignore_index, reduction="sum") / n.to(logits.dtype)
    conf = torch.from_numpy(O.confusion(logits.detach(), y_loc, K, ignore_index))
    dist.all_reduce(conf)
    dice = O.macro_dice_loss(conf.numpy(), K)
    ce_loc.backward()
    ce = ce_loc.detach().clone()
    dist.all_reduce(ce)
    for p in P.values():
        if p.grad is not None:
            dist.all_reduce(p.grad)
    return float(ce) + 0.5 * dice, float(ce), dice
