"""Depth-sharded engine (BASELINE config 4 path, include/spff.h shard_world /
shard_rank + spff_coll) on ONE GPU: 2 and 4 ranks, each its own process and
plan, exchange halos and all-reduce through host-staged gloo
(innovative3D.sharded.TorchDepthColl).  Their gathered logits, the loss and
the all-reduced gradients must match the unsharded engine on the same volume.
The 16-deep case gives each of 2 ranks 4 depth tiles, so the split-bf16 convs run
the halo exchange on the engine's side stream beside their interior depth tiles
(engine.hip conv_halo).  The height-sharded cases split the registry layout
[B, 1, 5, H, W] into row slabs (spff_cfg.shard_axis = SPFF_SHARD_HEIGHT,
innovative3D.sharded.HeightShardedSPFF); the full-size 1 x 1 x 5 x 512 x 512 registry
volume is checked against the kink-consistent oracle in test_gpu_baseline_sizes.py
(at 1.3 M voxels LeakyReLU / pool knife-edge flips move whole gradient tensors, so an
engine-vs-engine comparison there is not meaningful).  Marked gpu."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
K, BASE, SHAPE = 5, 8, (1, 5, 8, 32, 32)
# height-sharded cases: (batch, H, W, K, base) of the registry layout [B, 1, 5, H, W]
HCASES = {"small": (2, 32, 64, 5, 8)}


def _shape(depth):
    return (SHAPE[0], SHAPE[1], depth, SHAPE[3], SHAPE[4])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(math_mode, depth=SHAPE[2], k=K, base=BASE, in_ch=SHAPE[1]):
    import innovative3D.models as M
    from innovative3D.weightgen import synth_state
    core = M.build_spct_energyfilm_fourier(num_classes=k, base=base, in_channels=in_ch)
    for b in core._blocks():
        b.fgate._ensure_mask(depth, "cpu")
    st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=5)
    # a non-trivial FourierGate (mask / scale) so the sharded spectra matter
    for k in st:
        if k.endswith("freq_mask") or k.endswith("_mask"):
            st[k] = (0.5 + np.linspace(0, 1, st[k].size).reshape(st[k].shape)).astype(np.float32)
    core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    core = core.to("cuda")
    core.math = math_mode
    return core


def _data(depth=SHAPE[2]):
    from innovative3D.synthetic import synthetic_batch
    x, y = synthetic_batch(*_shape(depth), num_classes=K, ignore_frac=0.05, seed=11)
    return x, y


def _hdata(case):
    from innovative3D.synthetic import synthetic_batch
    B, H, W, k, _ = HCASES[case]
    return synthetic_batch(B, 1, 5, H, W, num_classes=k, ignore_frac=0.05, seed=13)


def _hworker(rank, world, port, math_mode, out, case, memory=None):
    import pathlib
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "spff-unet-spcct_amd")]
    from innovative3D.sharded import HeightShardedSPFF, height_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    B, H, W, k, base = HCASES[case]
    core = _model(math_mode, 5, k, base, 1)
    core.memory = memory
    x, y = _hdata(case)
    off, h = height_bounds(H, world, rank)
    step = HeightShardedSPFF(core, k, 255)
    loss, conf = step.step(x[:, :, :, off:off + h].contiguous().cuda(),
                           y[:, :, off:off + h].contiguous().cuda())
    torch.cuda.synchronize()
    np.savez(f"{out}.{rank}.npz", logits=step.last_logits.cpu().numpy(), loss=float(loss),
             conf=conf.cpu().numpy(),
             **{"g_" + kk: p.grad.cpu().numpy() for kk, p in core.named_parameters()
                if p.grad is not None})
    dist.barrier()
    dist.destroy_process_group()


def _worker(rank, world, port, math_mode, out, depth):
    import pathlib
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "spff-unet-spcct_amd")]
    from innovative3D.sharded import DepthShardedSPFF, shard_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    core = _model(math_mode, depth)
    x, y = _data(depth)
    off, d = shard_bounds(depth, world, rank)
    step = DepthShardedSPFF(core, K, 255)
    loss, conf = step.step(x[:, :, off:off + d].contiguous().cuda(), y[:, off:off + d].contiguous().cuda())
    torch.cuda.synchronize()
    np.savez(f"{out}.{rank}.npz", logits=step.last_logits.cpu().numpy(), loss=float(loss),
             conf=conf.cpu().numpy(),
             **{"g_" + k: p.grad.cpu().numpy() for k, p in core.named_parameters()
                if p.grad is not None})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,math_mode,depth", [
    (2, "f32", 8), (4, "f32", 8), (2, "bf16x6", 8), (4, "bf16x6", 8), (2, "bf16x6", 16)])
def test_depth_sharded_engine_matches_unsharded(tmp_path, world, math_mode, depth):
    import innovative3D.helpers as Hh
    core = _model(math_mode, depth)
    x, y = _data(depth)
    logits = core(x.cuda())
    loss, conf = Hh.ce_dice_with_confusion(logits, y.cuda(), K, 255)
    loss.backward()
    ref = logits.detach().cpu().numpy()
    grads = {k: p.grad.cpu().numpy() for k, p in core.named_parameters() if p.grad is not None}
    out = str(tmp_path / "sh")
    mp.spawn(_worker, args=(world, _free_port(), math_mode, out, depth), nprocs=world, join=True)
    parts = [np.load(f"{out}.{r}.npz") for r in range(world)]
    lg = np.concatenate([p["logits"] for p in parts], axis=2)
    e = float(np.abs(lg - ref).max())
    print(f"world {world} {math_mode} D {depth}: max|dlogit| {e:.2e}, loss {float(parts[0]['loss']):.7f} "
          f"vs {float(loss):.7f}")
    assert e <= 1e-4 * float(np.abs(ref).max())
    assert abs(float(parts[0]["loss"]) - float(loss)) <= 1e-5 * abs(float(loss))
    np.testing.assert_array_equal(parts[0]["conf"], conf.cpu().numpy())
    rows = []
    for k, g in grads.items():
        sc = max(float(np.abs(g).max()), 1e-30)
        eg = float(np.abs(parts[0]["g_" + k] - g).max()) / sc
        rows.append((eg, k))
        for p in parts[1:]:
            np.testing.assert_array_equal(p["g_" + k], parts[0]["g_" + k])
    rows.sort(reverse=True)
    print("  " + ", ".join(f"{k} {v:.1e}" for v, k in rows[:5]))
    bad = [(k, v) for v, k in rows if v > (5e-2 if k.endswith("mag_scale") else 2e-3)]
    assert not bad, bad


@pytest.mark.parametrize("world,math_mode,case,memory", [
    (2, "f32", "small", None), (4, "f32", "small", None), (2, "bf16x6", "small", None),
    (4, "bf16x6", "small", None),
    # the lean saved-activation layout (recomputed block outputs / decoder inputs)
    (2, "bf16x6", "small", "lean")])
def test_height_sharded_engine_matches_unsharded(tmp_path, world, math_mode, case, memory):
    import innovative3D.helpers as Hh
    B, H, W, k, base = HCASES[case]
    core = _model(math_mode, 5, k, base, 1)
    x, y = _hdata(case)
    logits = core(x.cuda())
    loss, conf = Hh.ce_dice_with_confusion(logits, y.cuda(), k, 255)
    loss.backward()
    ref = logits.detach().cpu().numpy()            # [B, K, D, H, W]
    grads = {kk: p.grad.cpu().numpy() for kk, p in core.named_parameters() if p.grad is not None}
    loss_ref, conf_ref = float(loss), conf.cpu().numpy()
    del core, logits, loss
    torch.cuda.empty_cache()
    out = str(tmp_path / "hsh")
    mp.spawn(_hworker, args=(world, _free_port(), math_mode, out, case, memory), nprocs=world,
             join=True)
    parts = [np.load(f"{out}.{r}.npz") for r in range(world)]
    lg = np.concatenate([p["logits"] for p in parts], axis=3)
    assert lg.shape == ref.shape, (lg.shape, ref.shape)
    e = float(np.abs(lg - ref).max())
    nflip = int((lg.argmax(1) != ref.argmax(1)).sum())
    print(f"H-shard world {world} {math_mode} {case} {memory or 'auto'}: max|dlogit| {e:.2e}, argmax flips {nflip}, "
          f"loss {float(parts[0]['loss']):.7f} vs {loss_ref:.7f}")
    assert e <= 1e-4 * float(np.abs(ref).max())
    assert abs(float(parts[0]["loss"]) - loss_ref) <= 1e-5 * abs(loss_ref)
    # the confusion counts match except where a logit within rounding of a tie flips
    assert int(np.abs(parts[0]["conf"] - conf_ref).sum()) <= 2 * nflip
    rows = []
    for kk, g in grads.items():
        sc = max(float(np.abs(g).max()), 1e-30)
        eg = float(np.abs(parts[0]["g_" + kk] - g).max()) / sc
        rows.append((eg, kk))
        for p in parts[1:]:
            np.testing.assert_array_equal(p["g_" + kk], parts[0]["g_" + kk])
    rows.sort(reverse=True)
    print("  " + ", ".join(f"{kk} {v:.1e}" for v, kk in rows[:5]))
    bad = [(kk, v) for v, kk in rows if v > (5e-2 if kk.endswith("mag_scale") else 2e-3)]
    assert not bad, bad
