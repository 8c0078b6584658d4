"""Host-side mirror checks (CPU): module tree / state-dict contract, registry,
metric algebra vs the oracle, and that the product path refuses CPU tensors."""
import math

import numpy as np
import pytest
import torch

from _golden import cfg_of, fixture_names, load
from _golden import build_core as _build_core
from oracle import spff_oracle as O
import innovative3D.config as C
import innovative3D.models as M
import innovative3D.helpers as Hh
from innovative3D import _engine as E


def _core_for(meta):
    return _build_core(meta)


@pytest.mark.parametrize("name", fixture_names())
def test_state_dict_keys_identical_to_reference(name):
    d = load(name)
    meta = d["meta"]
    if meta.get("lit"):
        mod = M.LitSPCT_EFiLM_FourierGate(num_classes=meta["K"])
        core = mod.model
    else:
        mod = core = _core_for(meta)
    D = d["x"].shape[2]
    for b in core._blocks():
        if isinstance(getattr(b, "fgate", None), M.FourierGate3D):
            b.fgate._ensure_mask(D, "cpu")
    sd = mod.state_dict()
    ref = d["state_shapes"]
    assert list(sd.keys()) == list(ref.keys())
    assert all(tuple(sd[k].shape) == tuple(v) for k, v in ref.items())
    # the lazily created mask is one tensor under two names (models.py:1532-1535)
    k = [k for k in sd if k.endswith("fgate._mask")]
    if k:
        fg = core.enc1.fgate
        assert fg._mask is fg.freq_mask


def test_registry_contract():
    names = [v[0] for v in C.VARIANTS]
    assert names[0] == "SPFF-UNet"
    for name, factory, dm, ckpt in C.VARIANTS:
        assert callable(factory) and callable(dm)
    lit = C.variant("SPFF-UNet")[1]()
    assert isinstance(lit, M.LitSPCT_EFiLM_FourierGate)
    assert lit.hparams.num_classes == C.NUM_CLASSES and lit.hparams.lr == C.BEST_LR
    assert sum(p.numel() for p in lit.parameters()) == 5491284


def test_selected_variant(monkeypatch):
    monkeypatch.setenv("INNOVATIVE3D_VARIANT", "SPFF-UNet")
    assert [v[0] for v in C.selected_variants()] == ["SPFF-UNet"]
    monkeypatch.setenv("INNOVATIVE3D_VARIANT", "nope")
    with pytest.raises(KeyError):
        C.selected_variants()


def test_cpu_tensors_are_refused():
    lit = M.LitSPCT_EFiLM_FourierGate(num_classes=9, base=8)
    with pytest.raises(E.SpffError):
        lit(torch.randn(1, 1, 5, 16, 16))
    with pytest.raises(E.SpffError):
        Hh.ce_plus_macro_dice_loss(torch.randn(1, 9, 5, 8, 8), torch.zeros(1, 5, 8, 8, dtype=torch.long), 9)


@pytest.mark.parametrize("name", fixture_names())
def test_metric_algebra_matches_reference(name):
    d = load(name)
    K = d["meta"]["K"]
    logits = torch.from_numpy(d["logits"])
    y = torch.from_numpy(d["labels"])
    conf = O.confusion(logits, y, K, 255)
    conf1 = np.concatenate([conf, np.zeros((K, 1), np.int64)], axis=1)  # no out-of-range labels
    met = Hh.metrics_from_confusion(conf1, K, y.numel())
    np.testing.assert_allclose(met[0], d["met_dice"], rtol=1e-12, equal_nan=True)
    np.testing.assert_allclose(met[1], d["met_sens"], rtol=1e-12, equal_nan=True)
    np.testing.assert_allclose(met[2], d["met_spec"], rtol=1e-12, equal_nan=True)
    np.testing.assert_allclose(met[3:], d["met_scalars"], rtol=1e-12, equal_nan=True)


def test_metric_algebra_ignore_none_with_255_labels():
    # ignore_index=None: label 255 is "some other class" for every c (helpers.py:675-678)
    torch.manual_seed(0)
    K = 5
    logits = torch.randn(1, K, 2, 4, 4)
    y = torch.randint(0, K, (1, 2, 4, 4))
    y[0, 0, 0, :] = 255
    pred = logits.argmax(1)
    conf = np.zeros((K, K + 1), np.int64)
    for p_, t_ in zip(pred.reshape(-1).tolist(), y.reshape(-1).tolist()):
        conf[p_, t_ if t_ < K else K] += 1
    met = Hh.metrics_from_confusion(conf, K, y.numel())
    # direct restatement of helpers.py:668-725 with mask = all-true
    for c in range(K):
        pc, lc = (pred == c), (y == c)
        tp = int((pc & lc).sum()); fp = int((pc & ~lc).sum()); fn = int((~pc & lc).sum())
        tn = int((~pc & ~lc).sum())
        spec = (tn + 1e-6) / (tn + fp + 1e-6)
        assert math.isclose(met[2][c], spec, rel_tol=1e-12)


def test_gate_settings_mirror():
    """EnergyFiLM3D(hidden, pe_dims) / FourierGate3D(learn_phase): accepted in the engine's
    range, one setting per network (include/spff.h spff_cfg.efilm_hidden ...)."""
    core = _core_for({"in_ch": 1, "K": 5, "base": 8})
    assert core._gate_settings() == {"efilm_hidden": 32, "efilm_pe_dims": 16,
                                     "fgate_learn_phase": False}
    for b in core._blocks():
        b.efilm = M.EnergyFiLM3D(b.efilm.channels, hidden=7, pe_dims=5)
        b.fgate = M.FourierGate3D(learn_phase=True)
    assert core._gate_settings() == {"efilm_hidden": 7, "efilm_pe_dims": 5,
                                     "fgate_learn_phase": True}
    assert tuple(core.enc1.efilm.mlp[0].weight.shape) == (7, 5, 1)
    core.enc2.fgate = M.FourierGate3D(learn_phase=False)
    with pytest.raises(NotImplementedError, match="same in every block"):
        core._gate_settings()
    for bad in ({"hidden": 65}, {"pe_dims": 1}, {"pe_dims": 33}, {"hidden": 0}):
        with pytest.raises(NotImplementedError, match="supports hidden"):
            M.EnergyFiLM3D(8, **bad)
