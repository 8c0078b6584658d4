#!/usr/bin/env python3
"""Per-layer conv3d kernel microbenchmark (fwd / dgrad / wgrad) at the SPFF-UNet
headline shapes (batch 2, 128^3, base 32).  Prints ms and TFLOP/s per op.

    python scripts/kbench.py [--ops fwd,dgrad,wgrad] [--iters 5] [--layers all|l0|...]
                             [--math f32|bf16x6|bf16x3]
"""
import argparse
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "spff-unet-spcct_amd")]

import torch  # noqa: E402

from innovative3D import _engine as E  # noqa: E402

# (name, level, cin, cout) of the 14 3x3x3 convs of SPFF-UNet (base 32, Cin 5)
LAYERS = [("enc1.pre", 0, 5, 32), ("enc1.body", 0, 32, 32), ("enc2.pre", 1, 32, 64),
          ("enc2.body", 1, 64, 64), ("enc3.pre", 2, 64, 128), ("enc3.body", 2, 128, 128),
          ("bott.pre", 3, 128, 256), ("bott.body", 3, 256, 256), ("dec3.pre", 2, 256, 128),
          ("dec3.body", 2, 128, 128), ("dec2.pre", 1, 128, 64), ("dec2.body", 1, 64, 64),
          ("dec1.pre", 0, 64, 32), ("dec1.body", 0, 32, 32)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--layers", default="all")
    ap.add_argument("--math", default="f32", choices=sorted(E.MATH_NAMES))
    args = ap.parse_args()
    L, p = E.lib(), E._ptr
    dev = torch.device("cuda", 0)
    st = E._stream(dev)
    ops = args.ops.split(",")
    m = E.MATH_NAMES[args.math]
    print(f"math={args.math}")
    tot = {o: [0.0, 0.0] for o in ops}
    for name, lvl, cin, cout in LAYERS:
        if args.layers != "all" and not name.startswith(args.layers):
            continue
        B, D, H, W = args.batch, args.size, args.size >> lvl, args.size >> lvl
        ldx = (cin + 7) // 8 * 8
        x = torch.randn(B, D, H, W, ldx, device=dev)
        w = torch.randn(cout, cin, 3, 3, 3, device=dev) * 0.05
        y = torch.empty(B, D, H, W, cout, device=dev)
        dx = torch.empty(B, D, H, W, cin, device=dev) if cin % 4 == 0 else None
        dw = torch.empty_like(w)
        ws = torch.empty(L.spff_conv3d_ws_bytes(B, D, H, W, cin, cout, 3), dtype=torch.uint8,
                         device=dev)
        flops = 2.0 * B * D * H * W * cin * cout * 27
        calls = {
            "fwd": lambda: L.spff_conv3d_fwd_ex(p(x), ldx, p(w), p(y), B, D, H, W, cin, cout, 3, m,
                                                p(ws), st),
            "dgrad": (lambda: L.spff_conv3d_dgrad_ex(p(y), p(w), p(dx), B, D, H, W, cin, cout, 3, m,
                                                     p(ws), st))
            if dx is not None else None,
            "wgrad": lambda: L.spff_conv3d_wgrad_ex(p(x), ldx, p(y), p(dw), B, D, H, W, cin, cout, 3, m,
                                                    p(ws), st),
        }
        row = []
        for o in ops:
            fn = calls[o]
            if fn is None:
                row.append(f"{o:>5}:    -    ")
                continue
            E.check(fn(), o)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                fn()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.iters
            tot[o][0] += ms
            tot[o][1] += flops
            row.append(f"{o:>5}: {ms:7.3f} ms {flops / ms / 1e9:6.1f} TF")
        print(f"{name:10s} " + "  ".join(row), flush=True)
    print("total      " + "  ".join(f"{o:>5}: {v[0]:7.3f} ms {v[1] / v[0] / 1e9:6.1f} TF"
                                    for o, v in tot.items() if v[0] > 0))


if __name__ == "__main__":
    main()
