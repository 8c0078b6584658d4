#!/usr/bin/env python3
"""Evaluation entry point of the MI355X engine, mirroring the parts of the
reference's test.py that touch the model (test.py:98-113 checkpoint lookup,
548-579 state-dict key alignment, 208-243 per-class aggregation over seeds):

  for each variant in VARIANTS (INNOVATIVE3D_VARIANT honoured) and seed in SEEDS:
  load best-*.ckpt (newest) or last.ckpt from CHECKPOINT_DIR/<model>/seed<k>/,
  run the engine on the test volumes, write test_details.csv (per volume and
  class: dice / sensitivity / specificity from the fused confusion kernel), and
  aggregate mean +- std over seeds into analysis/per_class_summary.csv -- the
  table the reference turns into heatmaps.

Plots (heatmaps, Bland-Altman, overlays) are host-side matplotlib analytics
outside the engine's scope; every number they draw is in the CSVs written here.
"""
from __future__ import annotations

import argparse
import csv
import os
import pathlib
import statistics
import sys
from typing import Dict, Optional

HERE = pathlib.Path(__file__).resolve().parent
if str(HERE) not in sys.path:
    sys.path.insert(0, str(HERE))

import torch  # noqa: E402

from innovative3D import config as C  # noqa: E402
from innovative3D import helpers as Hh  # noqa: E402
from innovative3D import models as M  # noqa: E402
from innovative3D.synthetic import SyntheticSPCCT  # noqa: E402
from train import Settings, _build_lit  # noqa: E402


def find_best_or_last_ckpt(ckpt_dir: pathlib.Path, model: str, seed: int) -> Optional[pathlib.Path]:
    """test.py:105-111: newest best-*.ckpt, else last.ckpt."""
    root = ckpt_dir / model / f"seed{seed}"
    bests = sorted(root.glob("best-*.ckpt"), key=lambda p: p.stat().st_mtime, reverse=True)
    if bests:
        return bests[0]
    p = root / "last.ckpt"
    return p if p.exists() else None


def align_state_dict_keys(ckpt_sd: Dict, model_sd: Dict) -> Dict:
    """test.py:548-579: add / strip the "model." and "module." prefixes so a
    checkpoint of the core loads into the Lit wrapper and vice versa."""
    def frac(keys, p):
        ks = [k for k in keys if "." in k]
        return sum(k.startswith(p) for k in ks) / max(1, len(ks)) if ks else 0.0

    for p in ("model.", "module."):
        want, have = frac(list(model_sd), p) > 0.9, frac(list(ckpt_sd), p) > 0.9
        if want and not have:
            ckpt_sd = {(k if k.startswith(p) else p + k): v for k, v in ckpt_sd.items()}
        elif have and not want:
            ckpt_sd = {(k[len(p):] if k.startswith(p) else k): v for k, v in ckpt_sd.items()}
    return ckpt_sd


def materialize_lazy(model, depth, device):
    """FourierGate masks are created lazily at the first forward (models.py:1527-
    1533); create them at the run's depth so a checkpoint that holds
    them loads strictly."""
    for m in model.modules():
        if isinstance(m, M.FourierGate3D):
            m._ensure_mask(depth, device)


def evaluate(model, dataset, K, device):
    rows = []
    model.eval()
    with torch.no_grad():
        for i in range(len(dataset)):
            x, y = dataset[i]
            x, y = x[None].to(device), y[None].to(device)
            logits = model(x)
            dice, sens, spec, *_ = Hh.per_class_metrics_3d(logits, y, K, ignore_index=255)
            for c in range(K):
                rows.append({"volume": i, "class": c, "dice": dice[c], "sens": sens[c],
                             "spec": spec[c]})
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="analysis")
    args = ap.parse_args(argv)
    S = Settings()
    device = torch.device("cuda", torch.cuda.current_device())
    out = pathlib.Path(args.out)
    out.mkdir(parents=True, exist_ok=True)
    summary = {}
    for name, builder, _dm, _base in C.selected_variants():
        for seed in S.seeds:
            ck = find_best_or_last_ckpt(S.ckpt_dir, name, seed)
            if ck is None:
                print(f"[test] {name} seed{seed}: no checkpoint under {S.ckpt_dir}")
                continue
            model = _build_lit(builder, S.in_ch).to(device)
            materialize_lazy(model, S.depth, device)
            sd = torch.load(ck, map_location="cpu", weights_only=True)
            sd = sd.get("state_dict", sd)
            model.load_state_dict(align_state_dict_keys(sd, model.state_dict()))
            K = int(model.hparams.num_classes)
            ds = SyntheticSPCCT(n=S.n_test, in_ch=S.in_ch, depth=S.depth, height=S.height,
                                width=S.width, num_classes=K, seed=seed + 20_000)
            rows = evaluate(model, ds, K, device)
            det = ck.parent / "test_details.csv"
            with open(det, "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=["volume", "class", "dice", "sens", "spec"])
                w.writeheader()
                w.writerows(rows)
            for c in range(K):
                vals = [r["dice"] for r in rows if r["class"] == c and r["dice"] == r["dice"]]
                if vals:
                    summary.setdefault((name, c), []).append(statistics.fmean(vals))
            print(f"[test] {name} seed{seed}: {ck.name} -> {det}")
    with open(out / "per_class_summary.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["model", "class", "dice_mean", "dice_std", "n_seeds"])
        for (name, c), v in sorted(summary.items()):
            w.writerow([name, c, statistics.fmean(v), statistics.pstdev(v) if len(v) > 1 else 0.0,
                        len(v)])
    print(f"[test] wrote {out / 'per_class_summary.csv'}")


if __name__ == "__main__":
    main()
