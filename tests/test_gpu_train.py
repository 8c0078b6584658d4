"""End-to-end entry points on the GPU: spff-unet-spcct_amd/train.py (two short
epochs of the SPFF-UNet variant with checkpoints, CSV logs, early-stopping
bookkeeping and the final test) and test.py (best-checkpoint reload, key
alignment, per-class summary).  Marked gpu."""
import csv
import math
import pathlib
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "spff-unet-spcct_amd"


def test_train_then_test(tmp_path, monkeypatch):
    env = {"CHECKPOINT_DIR": str(tmp_path / "ck"), "SEEDS": "7", "MAX_EPOCHS": "2",
           "BATCH_SIZE": "2", "NUM_FRAMES": "8", "IMAGE_HEIGHT": "32", "IMAGE_WIDTH": "32",
           "IN_CHANNELS": "5", "N_TRAIN": "4", "N_VAL": "2", "N_TEST": "2",
           "INNOVATIVE3D_VARIANT": "SPFF-UNet,PlainCore_UNet"}
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.syspath_prepend(str(PKG))
    sys.modules.pop("train", None)
    sys.modules.pop("test", None)
    import train as T
    res = T.main([])
    assert [r["model"] for r in res] == ["SPFF-UNet", "PlainCore_UNet"]
    for r in res:
        assert 0.0 <= r["test_macro_dice"] <= 1.0
        run = tmp_path / "ck" / r["model"] / "seed7"
        assert (run / "last.ckpt").exists()
        assert list(run.glob("best-*.ckpt"))
        rows = list(csv.DictReader(open(run / "logs" / "metrics.csv")))
        assert len(rows) == 2 and all(math.isfinite(float(x["train_loss"])) for x in rows)
        sd = torch.load(run / "last.ckpt", map_location="cpu", weights_only=True)["state_dict"]
        assert any(k.startswith("model.") for k in sd)
    assert (tmp_path / "ck" / "all_results.csv").exists()
    import test as TT
    # a checkpoint without the Lightning "model." prefix must load too
    run = tmp_path / "ck" / "SPFF-UNet" / "seed7"
    best = sorted(run.glob("best-*.ckpt"))[0]
    sd = torch.load(best, map_location="cpu", weights_only=True)
    sd["state_dict"] = {k[len("model."):]: v for k, v in sd["state_dict"].items()}
    torch.save(sd, best)
    TT.main(["--out", str(tmp_path / "analysis")])
    summ = list(csv.DictReader(open(tmp_path / "analysis" / "per_class_summary.csv")))
    assert {r["model"] for r in summ} == {"SPFF-UNet", "PlainCore_UNet"}
    assert (run / "test_details.csv").exists()
