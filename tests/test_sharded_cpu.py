"""Depth sharding (BASELINE config 4) and height sharding of
the registry layout on CPU with gloo: world sizes 2 and 4 run the sharded
restatement (oracle/spff_sharded.py) on slabs of one volume; the gathered logits, the loss and the all-reduced
gradients must equal the unsharded oracle's (fp64, 1e-9).  This pins the
exchange plan the engine's sharded plans implement: conv halos, distributed
InstanceNorm / SE statistics, the FourierGate all-gather, global-D EFiLM
encodings and the global CE normalisation."""
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


def _worker(rank, world, port, name, out_path, axis=2):
    import pathlib
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root / "tests"), str(root), str(root / "spff-unet-spcct_amd")]
    from _golden import cfg_of, load, state_of
    from oracle import spff_oracle as O
    from oracle import spff_sharded as S
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    d = load(name)
    cfg = cfg_of(d["meta"])
    P = O.params_from_state(state_of(d), dtype=torch.float64)
    sh = S.Shard(d["x"].shape[axis], rank, world, axis)
    x = torch.from_numpy(d["x"]).double().narrow(axis, sh.off, sh.D_loc).contiguous()
    y = torch.from_numpy(d["labels"]).narrow(axis - 1, sh.off, sh.D_loc).contiguous()
    with torch.no_grad():
        lg = S.forward(P, x, cfg, sh)
    loss, ce, dice = S.fwd_bwd(P, x, y, cfg, sh)
    np.savez(f"{out_path}.{rank}.npz", logits=lg.numpy(), loss=loss, ce=ce, dice=dice,
             **{"g_" + k: v.grad.numpy() for k, v in P.items() if v.grad is not None})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,world,axis", [
    ("fx3_fgate_even_b2", 2, 2), ("fx3_fgate_even_b2", 4, 2),
    ("fx2_ns_base8", 2, 2), ("fx2_ns_base8", 4, 2),
    # height sharding of the registry layout [B, 1, 5, H, W]
    ("fx1_registry_k13", 2, 3), ("fx1_registry_k13", 4, 3), ("fx3b_fgate_odd_b2", 2, 3),
    ("fx2_ns_base8", 2, 3)])
def test_sharded_equals_unsharded(tmp_path, name, world, axis):
    from oracle import spff_oracle as O
    d = load(name)
    cfg = cfg_of(d["meta"])
    P = O.params_from_state(state_of(d), dtype=torch.float64)
    x = torch.from_numpy(d["x"]).double()
    y = torch.from_numpy(d["labels"])
    K = d["meta"]["K"]
    logits = O.forward(P, x, cfg)
    ce = F.cross_entropy(logits, y, ignore_index=255)
    dice = O.macro_dice_loss(O.confusion(logits.detach(), y, K, 255), K)
    ce.backward()
    out = str(tmp_path / "sh")
    mp.spawn(_worker, args=(world, _free_port(), name, out, axis), nprocs=world, join=True)
    parts = [np.load(f"{out}.{r}.npz") for r in range(world)]
    lg = np.concatenate([p["logits"] for p in parts], axis=axis)
    ref = logits.detach().numpy()
    assert np.abs(lg - ref).max() <= 1e-9 * np.abs(ref).max()
    assert abs(float(parts[0]["ce"]) - float(ce)) <= 1e-12 * abs(float(ce))
    assert abs(float(parts[0]["dice"]) - dice) <= 1e-12
    for k, v in P.items():
        if v.grad is None:
            continue
        g = parts[0]["g_" + k]
        sc = max(float(v.grad.abs().max()), 1e-30)
        assert np.abs(g - v.grad.numpy()).max() <= 1e-9 * sc, k
        for p in parts[1:]:   # every rank holds the same all-reduced gradient
            np.testing.assert_array_equal(p["g_" + k], g)
