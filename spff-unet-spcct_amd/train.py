#!/usr/bin/env python3
"""Training entry point of the MI355X engine, mirroring the reference's
train.py (train_and_log / main, train.py:1398-1624) for the SPFF path:

  for each (name, builder, DataModule, base) in VARIANTS (config.py, honouring
  INNOVATIVE3D_VARIANT) and each seed: seed_everything -> build the Lit module
  -> Adam + ReduceLROnPlateau(mode=max on val_macro_dice) from the module's own
  configure_optimizers -> epochs of training_step / validation_step -> last.ckpt
  every epoch, best-{epoch}-{val_macro_dice}.ckpt on improvement, EarlyStopping
  (val_macro_dice, patience 12, min_delta 1e-3) -> test on the best weights ->
  logs/metrics.csv per run and all_results.csv over runs.

The Lightning Trainer is replaced by this loop (pytorch_lightning is not part of
the hot path, and not installed here); checkpoints keep Lightning's layout
({"state_dict": {"model....": ...}, "epoch": ...}) so they load into the
reference's modules and back.  Data: the DICOM MultiDicomDataModule3D is outside
the engine's scope; this driver feeds SyntheticSPCCT volumes of
the configured shape, or any Dataset passed to train_and_log().

Environment (defaults = the registry's constants, config.py): CHECKPOINT_DIR,
SEEDS ("42,123,999"), MAX_EPOCHS, BATCH_SIZE, NUM_FRAMES (depth), IMAGE_HEIGHT,
IMAGE_WIDTH, IN_CHANNELS (1 = registry layout, 5 = north-star layout),
N_TRAIN / N_VAL / N_TEST (synthetic volumes), FAST_TEST / --fast (one short
epoch of FAST_TEST_LIMIT batches), SPFF_MATH (conv arithmetic).
"""
from __future__ import annotations

import argparse
import csv
import math
import os
import pathlib
import sys
import time

HERE = pathlib.Path(__file__).resolve().parent
if str(HERE) not in sys.path:
    sys.path.insert(0, str(HERE))

import torch  # noqa: E402

from innovative3D import _engine as E  # noqa: E402
from innovative3D import config as C  # noqa: E402
from innovative3D.lightning_compat import pl  # noqa: E402
from innovative3D.synthetic import SyntheticSPCCT  # noqa: E402


def _env_int(name, default):
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


def _env_flag(name, default="0"):
    return os.environ.get(name, default).strip().lower() in ("1", "true", "yes", "on")


class Settings:
    """Run settings: the registry's constants (config.py) unless overridden by
    the environment.  The registry layout is [B, 1, NUM_FRAMES, H, W] (energy
    bins on depth); IN_CHANNELS=5 with NUM_FRAMES=D selects the north-star
    5-bins-as-channels layout."""

    def __init__(self):
        self.ckpt_dir = pathlib.Path(os.environ.get("CHECKPOINT_DIR", str(C.CHECKPOINT_DIR)))
        self.seeds = [int(s) for s in os.environ.get("SEEDS", ",".join(map(str, C.SEEDS))).split(",")
                      if s.strip()]
        self.max_epochs = _env_int("MAX_EPOCHS", C.FINAL_EPOCHS)
        self.batch = _env_int("BATCH_SIZE", C.BATCH_SIZE)
        self.depth = _env_int("NUM_FRAMES", C.NUM_FRAMES)
        self.height = _env_int("IMAGE_HEIGHT", C.IMAGE_HEIGHT)
        self.width = _env_int("IMAGE_WIDTH", C.IMAGE_WIDTH)
        self.in_ch = _env_int("IN_CHANNELS", 1)
        self.n_train = _env_int("N_TRAIN", 8)
        self.n_val = _env_int("N_VAL", 2)
        self.n_test = _env_int("N_TEST", 2)
        self.fast = _env_flag("FAST_TEST")
        self.fast_limit = _env_int("FAST_TEST_LIMIT", 2)
        self.patience = _env_int("EARLY_STOP_PATIENCE", 12)


def _build_lit(builder, in_ch):
    """train.py:1251-1270: a VARIANTS entry is a Lit class or a factory; the
    engine's factories take the input-channel count of the north-star layout."""
    try:
        return builder(in_channels=in_ch)
    except TypeError:
        return builder()


def _loader(ds, batch, shuffle, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.utils.data.DataLoader(ds, batch_size=batch, shuffle=shuffle, generator=g,
                                       drop_last=False)


def _scalar(v):
    return float(v.detach().float().mean()) if torch.is_tensor(v) else float(v)


def _run_epoch(model, loader, step_fn, limit, device, opt=None):
    """One pass; returns the batch-size-weighted mean of every logged metric."""
    sums, n = {}, 0
    model.train(opt is not None)
    for i, (x, y) in enumerate(loader):
        if limit and i >= limit:
            break
        x, y = x.to(device, non_blocking=True), y.to(device, non_blocking=True)
        model.logged_metrics = {}
        if opt is not None:
            opt.zero_grad(set_to_none=True)
            loss = step_fn((x, y), i)
            loss.backward()
            opt.step()
        else:
            with torch.no_grad():
                step_fn((x, y), i)
        bs = x.shape[0]
        for k, v in model.logged_metrics.items():
            v = _scalar(v)
            if not math.isnan(v):
                sums[k] = sums.get(k, 0.0) + v * bs
                sums[k + "#n"] = sums.get(k + "#n", 0) + bs
        n += bs
    return {k: sums[k] / sums[k + "#n"] for k in sums if not k.endswith("#n")}


def _save_ckpt(path, model, epoch, metrics):
    torch.save({"state_dict": {k: v.detach().cpu() for k, v in model.state_dict().items()},
                "epoch": epoch, "metrics": metrics}, path)


def train_and_log(model_name, builder, seed, S: Settings, datasets=None):
    """train.py:1398-1583 for one (variant, seed); returns test_macro_dice."""
    device = torch.device("cuda", torch.cuda.current_device())
    folder = S.ckpt_dir / model_name / f"seed{seed}"
    (folder / "logs").mkdir(parents=True, exist_ok=True)
    for p in folder.glob("last-v*.ckpt"):
        p.unlink()
    print(f"\n===== {model_name} | seed={seed} =====", flush=True)
    pl.seed_everything(seed, workers=True)
    model = _build_lit(builder, S.in_ch).to(device)
    if datasets is None:
        shape = dict(in_ch=S.in_ch, depth=S.depth, height=S.height, width=S.width,
                     num_classes=int(model.hparams.num_classes))
        datasets = (SyntheticSPCCT(n=S.n_train, seed=seed, **shape),
                    SyntheticSPCCT(n=S.n_val, seed=seed + 10_000, **shape),
                    SyntheticSPCCT(n=S.n_test, seed=seed + 20_000, **shape))
    tr, va, te = (_loader(d, S.batch, i == 0, seed) for i, d in enumerate(datasets))
    oc = model.configure_optimizers()
    if isinstance(oc, torch.optim.Optimizer):  # Lightning also accepts a bare optimizer (3DUNet)
        oc = {"optimizer": oc}
    opt = oc["optimizer"]
    sch = oc.get("lr_scheduler", {}).get("scheduler")
    monitor = oc.get("lr_scheduler", {}).get("monitor", "val_macro_dice")
    limit = S.fast_limit if S.fast else 0
    epochs = 1 if S.fast else S.max_epochs
    best, best_path, stale = -math.inf, None, 0
    rows = []
    for epoch in range(epochs):
        t0 = time.perf_counter()
        trm = _run_epoch(model, tr, model.training_step, limit, device, opt)
        vam = _run_epoch(model, va, model.validation_step, limit, device)
        score = vam.get(monitor, float("nan"))
        if sch is not None and not math.isnan(score):
            sch.step(score)
        row = {"epoch": epoch, "lr": opt.param_groups[0]["lr"], "sec": time.perf_counter() - t0,
               **trm, **vam}
        rows.append(row)
        print(f"[epoch {epoch}] train_loss {trm.get('train_loss', float('nan')):.4f} "
              f"val_loss {vam.get('val_loss', float('nan')):.4f} "
              f"val_macro_dice {score:.4f} ({row['sec']:.1f}s)", flush=True)
        _save_ckpt(folder / "last.ckpt", model, epoch, row)
        if not math.isnan(score) and score > best + 1e-3:
            best, stale = score, 0
            if best_path is not None and best_path.exists():
                best_path.unlink()
            best_path = folder / f"best-{epoch:02d}-{score:.4f}.ckpt"
            _save_ckpt(best_path, model, epoch, row)
        else:
            stale += 1
            if stale >= S.patience:
                print(f"[early stop] no val_macro_dice improvement in {S.patience} epochs")
                break
    keys = sorted({k for r in rows for k in r}, key=lambda k: (k not in ("epoch", "lr", "sec"), k))
    with open(folder / "logs" / "metrics.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=keys)
        w.writeheader()
        w.writerows(rows)
    if best_path is not None:
        sd = torch.load(best_path, map_location="cpu", weights_only=True)["state_dict"]
        model.load_state_dict(sd)
    tem = _run_epoch(model, te, model.test_step, limit, device)
    with open(folder / "test_metrics.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["metric", "value"])
        for k in sorted(tem):
            w.writerow([k, tem[k]])
    # free this run's engine plans / workspaces before the next (variant, seed)
    for m in model.modules():
        E.release_plans(m)
    return tem.get("test_macro_dice", float("nan"))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--fast", action="store_true", help="FAST_TEST=1: one short epoch")
    ap.add_argument("--fast-test-limit", type=int, default=None)
    args = ap.parse_args(argv)
    S = Settings()
    if args.fast:
        S.fast = True
        if args.fast_test_limit is not None:
            S.fast_limit = args.fast_test_limit
    S.ckpt_dir.mkdir(parents=True, exist_ok=True)
    results = []
    for name, builder, _dm, _base in C.selected_variants():
        for sd in S.seeds:
            results.append({"model": name, "seed": sd,
                            "test_macro_dice": train_and_log(name, builder, sd, S)})
    out = S.ckpt_dir / "all_results.csv"
    with open(out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["model", "seed", "test_macro_dice"])
        w.writeheader()
        w.writerows(results)
    print(f"\nSaved results to {out}")
    return results


if __name__ == "__main__":
    main()
