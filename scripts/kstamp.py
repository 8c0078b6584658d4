#!/usr/bin/env python3
"""Phase timing of k_conv3d_fwd_x from in-kernel timestamps (a variant library built
with -DSPFF_XSTAMP=1, selected by SPFF_LIB): per workgroup the s_memtime cycles of its
prologue (start -> first MFMA), k-loop and epilogue, and the launch's wall time.

    SPFF_LIB=abvar/libspff_xstamp.so python scripts/kstamp.py [--layers enc1.body,dec2.body]
"""
import argparse
import ctypes
import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "spff-unet-spcct_amd"), str(ROOT / "scripts")]

import torch  # noqa: E402

from innovative3D import _engine as E  # noqa: E402
from kbench import LAYERS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="enc1.body,enc2.body,dec1.body,dec2.pre")
    ap.add_argument("--ops", default="fwd,dgrad")
    ap.add_argument("--math", default="f16x3")
    args = ap.parse_args()
    L, p = E.lib(), E._ptr
    fn = L.spff_debug_xstamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    st = E._stream(dev)
    m = E.MATH_NAMES[args.math]
    N = 1 << 15
    buf = np.zeros((N, 16), dtype=np.uint64)
    for name, lvl, cin, cout in LAYERS:
        if name not in args.layers.split(","):
            continue
        B, D, H, W = 2, 128, 128 >> lvl, 128 >> lvl
        ldx = (cin + 7) // 8 * 8
        x = torch.randn(B, D, H, W, ldx, device=dev)
        w = torch.randn(cout, cin, 3, 3, 3, device=dev) * 0.05
        y = torch.empty(B, D, H, W, cout, device=dev)
        dx = torch.empty(B, D, H, W, cin, device=dev)
        ws = torch.empty(L.spff_conv3d_ws_bytes(B, D, H, W, cin, cout, 3), dtype=torch.uint8,
                         device=dev)
        for op in args.ops.split(","):
            call = ((lambda: L.spff_conv3d_fwd_ex(p(x), ldx, p(w), p(y), B, D, H, W, cin, cout, 3,
                                                  m, p(ws), st)) if op == "fwd" else
                    (lambda: L.spff_conv3d_dgrad_ex(p(y), p(w), p(dx), B, D, H, W, cin, cout, 3, m,
                                                    p(ws), st)))
            for _ in range(3):
                E.check(call(), op)
            torch.cuda.synchronize()
            buf[:] = 0
            assert L.spff_debug_xstamps_reset() == 0
            E.check(call(), op)
            torch.cuda.synchronize()
            assert fn(buf.ctypes.data, N) == 0
            t = buf[buf[:, 0] > 0].astype(np.int64)
            # keep only this launch: realtime window of the last launch
            r0, r1 = t[:, 4], t[:, 5]
            n = len(t)
            pro, loop, epi = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
            tot = t[:, 3] - t[:, 0]
            wall_us = (r1.max() - r0.min()) / 100.0  # s_memrealtime: 100 MHz
            cyc_per_us = float(np.median(tot / np.maximum((r1 - r0) / 100.0, 1e-3)))
            print(f"{name:10s} {op:5s} WGs {n:6d}  wall {wall_us:8.1f} us  clk {cyc_per_us:7.1f} MHz  "
                  f"per-WG us: prologue {np.median(pro) / cyc_per_us:6.2f}  k-loop "
                  f"{np.median(loop) / cyc_per_us:7.2f}  epilogue {np.median(epi) / cyc_per_us:6.2f}  "
                  f"total {np.median(tot) / cyc_per_us:7.2f} (p90 {np.percentile(tot, 90) / cyc_per_us:7.2f})",
                  flush=True)
            f = lambda a, b: np.median(t[:, b] - t[:, a]) / cyc_per_us  # noqa: E731
            print(f"{'':10s} {'':5s} prologue: fetch+prep {f(0, 8):5.2f}  scale barrier {f(8, 9):5.2f}  "
                  f"split+stash {f(9, 10):5.2f}  barrier B {f(10, 1):5.2f} | chunk 1: "
                  f"rescale+barrier A {f(11, 12):5.2f}  stash {f(12, 13):5.2f}  barrier B {f(13, 14):5.2f}  "
                  f"(chunk 0 body {f(1, 11):5.2f})", flush=True)
            # occupancy: average number of WGs in flight over the launch
            busy = (r1 - r0).sum() / 100.0
            print(f"{'':10s} {'':5s} mean WGs in flight {busy / wall_us:7.1f}  "
                  f"(sum of WG spans {busy:.0f} us); first start -> last start "
                  f"{(r0.max() - r0.min()) / 100.0:.1f} us", flush=True)


if __name__ == "__main__":
    main()
