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
