#!/usr/bin/env python3
"""Diagnostics for the conv arithmetics: (1) error statistics (max and mean
signed, i.e. bias) of the split-bf16 conv fwd/dgrad vs an fp64 conv, next to
the fp32 MFMA path; (2) on a golden fixture, f32 vs bf16x6 engine runs compared
stage by stage and gradient by gradient.

    python scripts/dbg_math.py [--fixture fx1_registry_k13]
"""
import argparse
import math
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "spff-unet-spcct_amd"), str(ROOT / "tests")]

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from innovative3D import _engine as E  # noqa: E402

DEV = "cuda"


def cl(t):
    return t.permute(0, 2, 3, 4, 1).contiguous()


def conv_stats(B, D, H, W, cin, cout, ksd=3, seed=3):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, cin, D, H, W, generator=g)
    w = torch.randn(cout, cin, ksd, 3, 3, generator=g) / math.sqrt(cin * ksd * 9)
    dy = torch.randn(B, cout, D, H, W, generator=g)
    y64 = cl(F.conv3d(x.double(), w.double(), None, padding=(ksd // 2, 1, 1)))
    dx64 = cl(torch.nn.grad.conv3d_input(x.shape, w.double(), dy.double(), padding=(ksd // 2, 1, 1)))
    ldx = (cin + 7) // 8 * 8
    xcl = torch.zeros(B, D, H, W, ldx)
    xcl[..., :cin] = cl(x)
    xcl, wd, dyg = xcl.to(DEV), w.to(DEV), cl(dy).to(DEV)
    L, p, st = E.lib(), E._ptr, E._stream(torch.device(DEV))
    ws = torch.empty(L.spff_conv3d_ws_bytes(B, D, H, W, cin, cout, ksd), dtype=torch.uint8, device=DEV)
    for name, m in E.MATH_NAMES.items():
        yg = torch.empty(B, D, H, W, cout, device=DEV)
        E.check(L.spff_conv3d_fwd_ex(p(xcl), ldx, p(wd), p(yg), B, D, H, W, cin, cout, ksd, m, p(ws), st), "f")
        row = []
        e = yg.cpu().double() - y64
        row.append(f"fwd max {e.abs().max() / y64.abs().max():.2e} rms {e.pow(2).mean().sqrt() / y64.pow(2).mean().sqrt():.2e} "
                   f"bias {(e * y64.sign()).mean() / y64.abs().mean():+.2e}")
        if cin % 4 == 0:
            dxg = torch.empty(B, D, H, W, cin, device=DEV)
            E.check(L.spff_conv3d_dgrad_ex(p(dyg), p(wd), p(dxg), B, D, H, W, cin, cout, ksd, m, p(ws), st), "d")
            e = dxg.cpu().double() - dx64
            row.append(f"dgrad max {e.abs().max() / dx64.abs().max():.2e} rms {e.pow(2).mean().sqrt() / dx64.pow(2).mean().sqrt():.2e} "
                       f"bias {(e * dx64.sign()).mean() / dx64.abs().mean():+.2e}")
        torch.cuda.synchronize()
        print(f"  [{B},{D},{H},{W}] {cin:3d}->{cout:3d} {name:7s} " + " | ".join(row), flush=True)


def fixture_compare(name):
    from _golden import load, state_of  # noqa: F401
    from test_gpu_parity import load_core
    import innovative3D.helpers as Hh
    d = load(name)
    K = d["meta"]["K"]
    res = {}
    for m in ("f32", "bf16x6", "bf16x3"):
        core = load_core(d)
        core.math = m
        x = torch.from_numpy(d["x"]).to(DEV)
        y = torch.from_numpy(d["labels"]).to(DEV)
        logits = core(x)
        loss, _ = Hh.ce_dice_with_confusion(logits, y, K, 255)
        loss.backward()
        torch.cuda.synchronize()
        grads = {k: v.grad.detach().double().cpu() for k, v in core.named_parameters() if v.grad is not None}
        stages = {}
        for blk in ("enc1", "enc2", "enc3", "bott", "dec3", "dec2", "dec1"):
            for s in ("y1", "y2", "out"):
                try:
                    stages[f"{blk}.{s}"] = core._plan.saved(f"{blk}.{s}").double().cpu()
                except Exception:
                    pass
        res[m] = (grads, stages)
    g32, s32 = res["f32"]
    for m in ("bf16x6", "bf16x3"):
        gm, sm = res[m]
        print(f"--- {name}: {m} vs f32")
        rows = []
        for k in s32:
            a, b = s32[k], sm[k]
            rows.append((float((a - b).abs().max() / a.abs().max().clamp_min(1e-30)), k))
        print("  stages: " + ", ".join(f"{k} {e:.1e}" for e, k in rows))
        rows = []
        for k in g32:
            a, b = g32[k], gm[k]
            rows.append((float((a - b).abs().max() / a.abs().max().clamp_min(1e-30)), k,
                         float(a.abs().max())))
        rows.sort(reverse=True)
        for e, k, mx in rows[:8]:
            print(f"  grad {k:34s} rel {e:.2e}  max|g| {mx:.3e}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fixture", default="fx1_registry_k13")
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--dskip", action="store_true")
    ap.add_argument("--perturb", action="store_true")
    args = ap.parse_args()
    if not args.no_stats:
        print("conv error statistics vs fp64 (relative to max / rms / mean|ref|):")
        for shp in [(1, 5, 32, 32, 8, 32), (1, 5, 32, 32, 32, 32), (1, 5, 32, 32, 64, 32),
                    (1, 5, 16, 16, 64, 64), (2, 16, 64, 64, 32, 32), (1, 8, 64, 64, 64, 64)]:
            conv_stats(*shp)
    if args.dskip:
        dskip_compare(args.fixture)
        return
    if args.perturb:
        perturb_sensitivity(args.fixture, math_mode="f32")
        perturb_sensitivity(args.fixture, math_mode="bf16x6")
        return
    import os
    print(f"SPFF_DEBUG_SPLIT={os.environ.get('SPFF_DEBUG_SPLIT', '')}")
    fixture_compare(args.fixture)



def dskip_compare(name="fx1_registry_k13"):
    """Engine (f32 / bf16x6) gradient at the encoder outputs vs the fp64 oracle
    run with that engine's own LeakyReLU signs and pool argmaxes."""
    from _golden import load, state_of, cfg_of
    from test_gpu_parity import load_core, engine_lrelu_masks
    from oracle import spff_oracle as O
    import innovative3D.helpers as Hh
    d = load(name)
    K, B = d["meta"]["K"], d["x"].shape[0]
    cfg = cfg_of(d["meta"])
    Dd, H0, W0 = d["x"].shape[2:]
    for m in ("f32", "bf16x6"):
        core = load_core(d)
        core.math = m
        x = torch.from_numpy(d["x"]).to(DEV)
        y = torch.from_numpy(d["labels"]).to(DEV)
        logits = core(x)
        loss, _ = Hh.ce_dice_with_confusion(logits, y, K, 255)
        loss.backward()
        torch.cuda.synchronize()
        eng = {l: core._plan.saved(f"grad.dskip{l}").double().cpu() for l in range(3)}
        masks = engine_lrelu_masks(core, d)
        posts = []
        oc, op, opost = O.conv_in_lrelu, O.maxpool, O._post
        npool = [0]

        def hc(P_, pre, inp, ksd):
            yy = F.conv3d(inp, P_[pre + ".0.weight"], None, padding=(ksd // 2, 1, 1))
            r = F.instance_norm(yy, weight=P_[pre + ".1.weight"], bias=P_[pre + ".1.bias"], eps=1e-5)
            return torch.where(masks[pre], r, 0.01 * r)

        def hp(t):
            k = npool[0] % 3
            npool[0] += 1
            B_, C_, D_, H_, W_ = t.shape
            v = t.reshape(B_, C_, D_, H_ // 2, 2, W_ // 2, 2).permute(0, 1, 2, 3, 5, 4, 6)
            v = v.reshape(B_, C_, D_, H_ // 2, W_ // 2, 4)
            return v.gather(-1, masks[f"pool{k + 1}"].unsqueeze(-1)).squeeze(-1)

        def hpost(P_, xx, stage, cfg_):
            o = opost(P_, xx, stage, cfg_)
            o.retain_grad()
            posts.append(o)
            return o
        O.conv_in_lrelu, O.maxpool, O._post = hc, hp, hpost
        try:
            P = O.params_from_state(state_of(d), dtype=torch.float64)
            O.fwd_bwd(P, torch.from_numpy(d["x"]).double(), torch.from_numpy(d["labels"]), cfg)
        finally:
            O.conv_in_lrelu, O.maxpool, O._post = oc, op, opost
        for l in range(3):
            g = posts[l].grad  # [B, C, D, H, W]
            C = g.shape[1]
            ref = g.permute(0, 2, 3, 4, 1).reshape(-1, C)
            e = eng[l] - ref
            sc = ref.abs().max()
            per_d = e.view(B, Dd, H0 >> l, W0 >> l, C).pow(2).mean(dim=(0, 2, 3, 4)).sqrt() / sc
            print(f"  {name} {m:7s} dskip{l}: max {float(e.abs().max() / sc):.2e} "
                  f"rms {float(e.pow(2).mean().sqrt() / sc):.2e}  per-d rms "
                  + " ".join(f"{float(v):.1e}" for v in per_d), flush=True)



def perturb_sensitivity(name="fx1_registry_k13", eps=(1e-7, 3e-7), math_mode="f32"):
    """How far each gradient moves when the INPUT is perturbed at fp32-rounding
    scale: the conditioning every fp32 implementation is subject to."""
    from _golden import load
    from test_gpu_parity import load_core
    import innovative3D.helpers as Hh
    d = load(name)
    K = d["meta"]["K"]

    def grads(x_np):
        core = load_core(d)
        core.math = math_mode
        x = torch.from_numpy(x_np).to(DEV)
        y = torch.from_numpy(d["labels"]).to(DEV)
        logits = core(x)
        loss, _ = Hh.ce_dice_with_confusion(logits, y, K, 255)
        loss.backward()
        torch.cuda.synchronize()
        return {k: v.grad.detach().double().cpu() for k, v in core.named_parameters() if v.grad is not None}
    g0 = grads(d["x"])
    import numpy as np
    for e in eps:
        for seed in (1, 2, 3):
            rng = np.random.default_rng(seed)
            xp = (d["x"] * (1 + e * rng.standard_normal(d["x"].shape))).astype(np.float32)
            g1 = grads(xp)
            rows = sorted(((float((g1[k] - g0[k]).abs().max() / g0[k].abs().max()), k) for k in g0),
                          reverse=True)[:4]
            print(f"  {math_mode} input eps {e:.0e} seed {seed}: "
                  + ", ".join(f"{k} {v:.1e}" for v, k in rows), flush=True)


if __name__ == "__main__":
    main()
