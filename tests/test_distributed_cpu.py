"""World-size-2 gloo test of the data-parallel path (CPU).

Each rank runs the CPU oracle on its own sample with the CE normalised by the
GLOBAL valid count (innovative3D.distributed.global_valid_count) and
all-reduces the gradient (allreduce_gradients).  The result must equal the
single-process full-batch gradient -- the exactness argument the engine's DP
mode (bench.py --gpus N) relies on."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from _golden import cfg_of, load, state_of


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import sys
    import pathlib
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "tests"), str(root), str(root / "spff-unet-spcct_amd")]
    from _golden import cfg_of, load, state_of
    from oracle import spff_oracle as O
    from innovative3D import distributed as Dd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    d = load("fx3_fgate_even_b2")
    cfg = cfg_of(d["meta"])
    P = O.params_from_state(state_of(d), dtype=torch.float64)
    x = torch.from_numpy(d["x"][rank:rank + 1]).double()
    y = torch.from_numpy(d["labels"][rank:rank + 1])
    cnt = Dd.global_valid_count(y, 255, count_fn=lambda t, ig: (t != ig).sum().reshape(1))
    logits = O.forward(P, x, cfg)
    loss = F.cross_entropy(logits, y, ignore_index=255, reduction="sum") / cnt.double()
    loss.backward()
    Dd.allreduce_gradients(list(P.values()))
    if rank == 0:
        np.savez(out_path, **{k: v.grad.numpy() for k, v in P.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_dp_two_ranks_equals_full_batch(tmp_path):
    from oracle import spff_oracle as O
    d = load("fx3_fgate_even_b2")
    assert d["x"].shape[0] == 2
    out = str(tmp_path / "g.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    cfg = cfg_of(d["meta"])
    P = O.params_from_state(state_of(d), dtype=torch.float64)
    logits = O.forward(P, torch.from_numpy(d["x"]).double(), cfg)
    F.cross_entropy(logits, torch.from_numpy(d["labels"]), ignore_index=255).backward()
    got = np.load(out)
    for k, v in P.items():
        ref = v.grad.numpy()
        assert np.abs(got[k] - ref).max() <= 1e-10 * max(1.0, np.abs(ref).max()), k


def test_single_process_helpers_are_noops():
    from innovative3D import distributed as Dd
    p = torch.nn.Parameter(torch.ones(3))
    p.grad = torch.full((3,), 2.0)
    Dd.allreduce_gradients([p])
    assert torch.equal(p.grad, torch.full((3,), 2.0))
    c = Dd.global_valid_count(torch.tensor([1, 255, 3]), 255,
                              count_fn=lambda t, ig: (t != ig).sum().reshape(1))
    assert int(c) == 2


def _worker_loss(rank, world, port, out_path):
    """Per rank: the CE share (CE normalised by the global count) and confusion
    of its own sample -> distributed.global_loss; and a GradBucketer run over a
    flat vector with ranges reported in the engine's backward order."""
    import sys
    import pathlib
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "tests"), str(root), str(root / "spff-unet-spcct_amd")]
    from _golden import cfg_of, load, state_of
    from oracle import spff_oracle as O
    from innovative3D import distributed as Dd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    d = load("fx3_fgate_even_b2")
    cfg = cfg_of(d["meta"])
    K = cfg.num_classes
    P = O.params_from_state(state_of(d), requires_grad=False)
    x = torch.from_numpy(d["x"][rank:rank + 1])
    y = torch.from_numpy(d["labels"][rank:rank + 1])
    cnt = Dd.global_valid_count(y, 255, count_fn=lambda t, ig: (t != ig).sum().reshape(1))
    logits = O.forward(P, x, cfg)
    ce = F.cross_entropy(logits, y, ignore_index=255, reduction="sum") / cnt.double()
    conf = torch.zeros(K, K + 1, dtype=torch.int64)
    conf[:, :K] = torch.from_numpy(O.confusion(logits, y, K, 255))
    loss, ce_g, conf_g = Dd.global_loss(ce.float(), conf, K)
    # bucketed gradient all-reduce: rank-dependent values, engine-like range order
    n = 1000
    flat = torch.arange(n, dtype=torch.float32) * (rank + 1)
    b = Dd.GradBucketer(bucket_bytes=4 * 150)
    b.begin(flat)
    for a, m in ((900, 100), (700, 200), (650, 50), (990 - 990, 100), (300, 350), (100, 200)):
        b.ready(a, m)
    b.finish()
    if rank == 0:
        np.savez(out_path, loss=loss.numpy(), ce=ce_g.numpy(), conf=conf_g.numpy(),
                 flat=flat.numpy(), launched=np.array(b.launched))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_global_loss_and_bucketed_allreduce(tmp_path):
    """DataParallelSPFF semantics (SURVEY §8(e) DP row; helpers.py:782-803): the
    loss / confusion of a world-2 step equal the single-process full-batch
    values, and the bucketed all-reduce sums every float exactly once."""
    from oracle import spff_oracle as O
    d = load("fx3_fgate_even_b2")
    out = str(tmp_path / "l.npz")
    mp.spawn(_worker_loss, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    cfg = cfg_of(d["meta"])
    K = cfg.num_classes
    P = O.params_from_state(state_of(d), requires_grad=False)
    logits = O.forward(P, torch.from_numpy(d["x"]), cfg)
    y = torch.from_numpy(d["labels"])
    loss, ce, dice = O.ce_plus_macro_dice(logits, y, K)
    conf = O.confusion(logits, y, K, 255)
    assert np.array_equal(got["conf"][:, :K], conf) and not got["conf"][:, K].any()
    assert abs(float(got["ce"]) - float(ce)) <= 2e-7 * abs(float(ce))
    assert abs(float(got["loss"]) - float(loss)) <= 2e-7 * abs(float(loss))
    assert np.array_equal(got["flat"], np.arange(1000, dtype=np.float32) * 3)
    spans = sorted(map(tuple, got["launched"]))
    assert spans[0][0] == 0 and spans[-1][1] == 1000
    assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert len(spans) < 6  # adjacent ranges were merged into buckets


def test_dice_loss_from_confusion_t_matches_host():
    import innovative3D.helpers as Hh
    rng = np.random.default_rng(0)
    for K in (2, 9, 13):
        conf = rng.integers(0, 50, size=(K, K + 1))
        conf[rng.integers(0, K), :] = 0
        a = Hh.dice_loss_from_confusion(conf, K)
        b = float(Hh.dice_loss_from_confusion_t(torch.from_numpy(conf), K))
        assert abs(a - b) <= 1e-15


def _worker_timeout(rank, world, port, out_path):
    """rank 1 never joins the halo exchange: rank 0's host-staged TorchDepthColl must
    raise within its deadline (SURVEY §5 failure detection) instead of hanging."""
    import sys
    import pathlib
    import time
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "tests"), str(root), str(root / "spff-unet-spcct_amd")]
    from innovative3D.sharded import TorchDepthColl
    import datetime
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=60))
    coll = TorchDepthColl(timeout=2.0)
    msg = ""
    if rank == 0:
        slab = torch.zeros(4 * 8)
        t0 = time.time()
        try:
            coll.halo(slab, 8, 2)
        except RuntimeError as e:
            msg = str(e)
        np.savez(out_path, msg=np.array(msg), dt=np.array(time.time() - t0))
    else:
        time.sleep(6.0)   # a stalled peer: never posts its side of the exchange
    os._exit(0)           # skip the (now mismatched) process-group teardown


def test_host_staged_halo_times_out(tmp_path):
    out = str(tmp_path / "t.npz")
    mp.spawn(_worker_timeout, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    assert "did not complete within 2 s" in str(got["msg"]), str(got["msg"])
    assert float(got["dt"]) < 5.0


def test_data_parallel_hooks_every_submodule_and_falls_back(monkeypatch):
    """the grad hook must reach the module that calls the engine plan
    (``.backbone``, ``.model.model``), and a step in which no plan took it must still
    all-reduce the gradients (world > 1)."""
    from innovative3D import distributed as Dd
    import innovative3D.helpers as Hh

    seen = []

    class Inner(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.ones(3))

        def forward(self, x):
            seen.append(getattr(self, "grad_hook", None))
            return x * self.w

    class Outer(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.backbone = Inner()

        def forward(self, x):
            return self.backbone(x)

    m = Outer()
    calls = []
    monkeypatch.setattr(Dd, "world", lambda group=None: 2)
    monkeypatch.setattr(Dd, "global_valid_count", lambda *a, **k: None)
    monkeypatch.setattr(Dd, "allreduce_gradients", lambda params, group=None, **k: calls.append(1))
    monkeypatch.setattr(Dd, "global_loss", lambda ce, conf, K, group=None, **k: (ce, ce, conf))
    monkeypatch.setattr(Hh, "ce_dice_parts",
                        lambda lg, y, K, ig, count_override=None: (lg.sum(), None, lg.sum()))
    dp = Dd.DataParallelSPFF(m, 3)
    dp.step(torch.ones(3), None)
    assert seen and seen[0] is dp.bucketer          # reached the nested module
    assert getattr(m.backbone, "grad_hook", "x") is None   # and was removed afterwards
    assert calls == [1]                              # no plan began the hook: fallback ran
    assert torch.equal(m.backbone.w.grad, torch.ones(3))


def test_data_parallel_reduces_parameters_outside_the_plan(monkeypatch):
    """once an engine op takes the hook, the parameters it covered are
    reduced by the buckets, and every OTHER parameter (a wrapper's own, outside the
    plan's flat buffer) is still all-reduced after the backward -- exactly once."""
    from innovative3D import distributed as Dd
    import innovative3D.helpers as Hh

    class Plan(torch.nn.Module):     # stands in for an engine op: covers its parameter
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.ones(3))

        def forward(self, x):
            hook = self.grad_hook
            hook.begin(torch.zeros(3))
            hook.cover([id(self.w)])
            return x * self.w

    class Wrapper(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.core = Plan()
            self.extra = torch.nn.Parameter(torch.full((2,), 2.0))

        def forward(self, x):
            return self.core(x) * self.extra.sum()

    m = Wrapper()
    reduced = []
    monkeypatch.setattr(Dd, "world", lambda group=None: 2)
    monkeypatch.setattr(Dd, "global_valid_count", lambda *a, **k: None)
    monkeypatch.setattr(Dd, "allreduce_gradients",
                        lambda params, group=None, **k: reduced.append([id(p) for p in params]))
    monkeypatch.setattr(Dd, "global_loss", lambda ce, conf, K, group=None, **k: (ce, ce, conf))
    monkeypatch.setattr(Hh, "ce_dice_parts",
                        lambda lg, y, K, ig, count_override=None: (lg.sum(), None, lg.sum()))
    dp = Dd.DataParallelSPFF(m, 3)
    dp.step(torch.ones(3), None)
    assert reduced == [[id(m.extra)]]
    # a second step starts from an empty coverage set
    reduced.clear()
    dp.step(torch.ones(3), None)
    assert reduced == [[id(m.extra)]]


def test_sharded_overlap_default(monkeypatch):
    """the sharded runners overlap the bucketed gradient all-reduces with
    the backward by default only when the halo collectives are host-staged (the tested path);
    device (RCCL) collectives need SPFF_SHARD_OVERLAP=1 until a multi-GPU run has exercised
    them (innovative3D/sharded.py _default_overlap)."""
    from innovative3D.sharded import _default_overlap

    class Coll:
        def __init__(self, host):
            self.host = host

    monkeypatch.delenv("SPFF_SHARD_OVERLAP", raising=False)
    assert _default_overlap(Coll(True)) is True
    assert _default_overlap(Coll(False)) is False
    assert _default_overlap(object()) is True  # a custom coll without the attribute
    monkeypatch.setenv("SPFF_SHARD_OVERLAP", "1")
    assert _default_overlap(Coll(False)) is True
