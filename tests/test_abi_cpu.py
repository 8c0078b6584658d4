"""CPU-only checks of the C-ABI library and the host-side mirror (no GPU calls)."""
import ctypes
import pathlib
import re

import numpy as np
import pytest
import torch

from _golden import cfg_of, fixture_names, load
from innovative3D import _engine as E

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _header_symbols():
    src = (ROOT / "include" / "spff.h").read_text()
    return sorted(set(re.findall(r"\b(spff_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    L = E.lib()
    syms = _header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(E.EXPORTED)


def test_plan_layout_matches_reference_state_dict():
    for name in fixture_names():
        d = load(name)
        m = d["meta"]
        cfg = cfg_of(m)
        x = d["x"]
        B, Cin, D, H, W = x.shape
        plan = E.Plan(B, Cin, D, H, W, cfg.num_classes, base=cfg.base, ksd=3, efilm=cfg.efilm,
                      fgate=cfg.fgate, se=cfg.se, specse=cfg.specse, efilm_hidden=cfg.efilm_hidden,
                      efilm_pe_dims=cfg.efilm_pe_dims, fgate_learn_phase=cfg.learn_phase)
        prefix = "model." if m.get("lit") else ""
        ref = {k[len(prefix):]: tuple(v) for k, v in d["state_shapes"].items()}
        ref_order = [k for k in ref if not k.endswith("._mask")]
        assert [p[0] for p in plan.params] == ref_order, name
        for pname, shape, off, n in plan.params:
            assert tuple(shape) == ref[pname]
            assert n == int(np.prod(shape))
        offs = [p[2] for p in plan.params]
        assert offs == sorted(offs) and plan.nfloats == offs[-1] + plan.params[-1][3]


def test_plan_rejects_bad_shapes():
    with pytest.raises(E.SpffError):
        E.Plan(1, 1, 5, 4, 64, 13)    # H < 8: three (1,2,2) pools
    # H, W not multiples of 8 take the _cat trilinear fallback (models.py:687-691)
    E.Plan(1, 1, 5, 60, 66, 13)
    with pytest.raises(E.SpffError):
        E.Plan(1, 1, 5, 64, 64, 129)  # K > SPFF_MAX_CLASSES
    with pytest.raises(E.SpffError):
        E.Plan(1, 1, 5, 64, 64, 13, base=20)  # base not a multiple of 8
    # the module contract beyond the registry settings (fixture fx5_k40_base24)
    p = E.Plan(1, 5, 6, 24, 24, 40, base=24)
    assert p.nfloats > 0 and p.ws_bytes > 0
    E.Plan(1, 72, 4, 16, 16, 128, base=40)


def test_workspace_size_headline_config_fits_hbm():
    p = E.Plan(2, 5, 128, 128, 128, 13)
    assert 5e9 < p.ws_bytes < 40e9
    # 5 491 284 (registry, Cin=1) + 27*32*4 (Cin=5 first conv) + 7 lazy masks of L=65
    assert p.nfloats == 5491284 + 27 * 32 * 4 + 7 * 65


def test_full_volume_512_fits_one_mi355x():
    """BASELINE configs[3]: one 1 x 5 x 512^3 volume on ONE GPU (the north star's
    8-vs-1 comparison on the same volume).  memory_mode auto picks the lean layout
    from 2^26 voxels; its workspace must leave room on 288 GB of HBM for the input
    (2.7 GB), labels (1.1 GB), logits and dlogits (7.0 GB each) and the flat params."""
    p = E.Plan(1, 5, 512, 512, 512, 13)
    V = 512 ** 3
    assert p.memory == "auto" and p.layout == "lean"
    assert p.ws_bytes / V <= 1750, p.ws_bytes / V
    assert p.ws_bytes + V * (5 * 4 + 8 + 2 * 13 * 4) < 250 * 2 ** 30
    full = E.Plan(1, 5, 512, 512, 512, 13, memory="full")
    assert full.ws_bytes > 288e9  # why the lean layout exists
    head = E.Plan(2, 5, 128, 128, 128, 13)  # the headline keeps the full (fastest) layout
    assert head.ws_bytes == E.Plan(2, 5, 128, 128, 128, 13, memory="full").ws_bytes
    with pytest.raises(E.SpffError):
        E.Plan(1, 5, 8, 32, 32, 5, memory="small")


def test_height_sharded_plan_shapes():
    """SPFF_SHARD_HEIGHT (registry layout [B, 1, 5, H, W]): local rows and
    width multiples of 8, any batch; the plan carries the row-padded conv operands on top
    of the unsharded layout of its slab, but no depth halos."""
    whole = E.Plan(1, 1, 5, 512, 512, 13)
    for world in (2, 4, 8):
        h = 512 // world
        p = E.Plan(2, 1, 5, h, 512, 13, shard_world=world, shard_rank=world - 1, shard_axis=1)
        assert p.nfloats == whole.nfloats  # same parameters (the FourierGate at D = 5)
        unsh = E.Plan(2, 1, 5, h, 512, 13)
        assert unsh.ws_bytes < p.ws_bytes < 1.6 * unsh.ws_bytes
    with pytest.raises(E.SpffError):
        E.Plan(1, 1, 5, 60, 512, 13, shard_world=2, shard_rank=0, shard_axis=1)  # 60 rows
    with pytest.raises(E.SpffError):
        E.Plan(1, 1, 5, 64, 512, 13, shard_world=2, shard_rank=0, shard_axis=2)  # bad axis
    with pytest.raises(E.SpffError):  # depth sharding keeps batch 1
        E.Plan(2, 1, 8, 64, 64, 13, shard_world=2, shard_rank=0, shard_axis=0)


def test_workspace_oom_releases_other_cached_plans(monkeypatch):
    """a workspace allocation that runs out of device memory releases the
    workspaces of the OTHER cached plans (their pending backward then fails loudly: the
    generation moves), empties torch's cache and retries once."""
    import types
    other = types.SimpleNamespace(ws_bytes=8, _ws=torch.empty(8, dtype=torch.uint8), generation=3)
    me = types.SimpleNamespace(ws_bytes=16, _ws=None, generation=0)
    monkeypatch.setitem(E._ANON_PLANS, ("other",), other)
    calls = []
    real_empty = torch.empty

    def fake_empty(*a, **k):
        calls.append(1)
        if len(calls) == 1:
            raise torch.OutOfMemoryError("simulated")
        return real_empty(*a, **{kk: v for kk, v in k.items() if kk != "device"})
    monkeypatch.setattr(torch, "empty", fake_empty)
    monkeypatch.setattr(torch.cuda, "empty_cache", lambda: None)
    ws = E._alloc_workspace(me, "cpu")
    assert ws.numel() == 16 and len(calls) == 2
    assert other._ws is None and other.generation == 4
