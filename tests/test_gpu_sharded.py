"""Depth-sharded engine (BASELINE config 4 path, include/spff.h shard_world /
shard_rank + spff_coll) on ONE GPU: 2 and 4 ranks, each its own process and
plan, exchange halos and all-reduce through host-staged gloo
(innovative3D.sharded.TorchDepthColl).  Their gathered logits, the loss and
the all-reduced gradients must match the unsharded engine on the same volume.
The 16-deep case gives each of 2 ranks 4 depth tiles, so the split-bf16 convs run
the halo exchange on the engine's side stream beside their interior depth tiles
(engine.hip conv_halo).

Gradients are judged BRANCH-CONSISTENTLY: against the fp64 oracle run with the
sharded engine's own LeakyReLU signs and max-pool argmaxes (each rank's slab,
gathered; test_gpu_parity.engine_branch_masks / oracle_grads_st), not against the
unsharded engine.  Two fp32 engines whose reductions sum in different orders may
put a LeakyReLU input that sits on its kink on opposite sides, which moves a
gradient tensor by up to 14 % at these tiny sizes (round 2: the 4-wave conv tiles'
fused statistics order) -- a legitimate fp32 outcome, not a sharding error.  The
logits, loss and confusion (robust to such flips) are still compared with the
unsharded engine.  The height-sharded cases split the registry layout
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
    core._synth_state = st
    return core


def _cfg(k=K, base=BASE, in_ch=SHAPE[1]):
    from oracle import spff_oracle as O
    return O.SpffCfg(in_ch=in_ch, num_classes=k, base=base)


def _save_masks(core, local_shape, cfg):
    """this rank's LeakyReLU signs / pool argmaxes over its own slab (npz-ready)"""
    from test_gpu_parity import engine_branch_masks
    masks = engine_branch_masks(core, local_shape, core._synth_state, cfg)
    mk = {}
    for kk, m in masks.items():
        a = m.numpy()
        mk["m_" + kk] = np.packbits(a) if a.dtype == np.bool_ else a.astype(np.uint8)
        mk["s_" + kk] = np.array(a.shape)
    return mk


def _gather_masks(parts, axis):
    """the ranks' branch decisions concatenated along the sharded axis (2 = D, 3 = H)"""
    masks = {}
    for kk in (f[2:] for f in parts[0].files if f.startswith("m_")):
        segs = []
        for p in parts:
            shp = tuple(int(v) for v in p["s_" + kk])
            a = p["m_" + kk]
            a = np.unpackbits(a)[:int(np.prod(shp))].astype(bool) if kk[:4] != "pool" else a
            segs.append(a.reshape(shp))
        cat = np.concatenate(segs, axis=axis)
        masks[kk] = (torch.from_numpy(cat) if cat.dtype == np.bool_
                     else torch.from_numpy(cat.astype(np.int64)))
    return masks


def _check_vs_oracle(parts, axis, st, cfg, x, y, mth, device="cpu"):
    """the sharded engine's gradients (rank 0; all ranks hold the same all-reduced
    gradient) vs the fp64 oracle with the sharded engine's own branch decisions
    (``device`` != "cpu": the fp64 oracle alone, evaluated there, floor tolerance)"""
    from test_gpu_parity import check_grads, oracle_grads_st
    masks = _gather_masks(parts, axis)
    ref64, ref32, nflip, absb = oracle_grads_st(cfg, st, x.numpy(), y.numpy(), masks,
                                                device=device, fp32=device == "cpu")
    print(f"  branch decisions differing from the fp64 oracle's own: {nflip}")
    check_grads({k: parts[0]["g_" + k] for k in ref64}, ref64, ref32, absb, st, mth)


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
    sys.path[:0] = [str(root), str(root / "tests"), str(root / "spff-unet-spcct_amd")]
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
    mk = _save_masks(core, (B, 1, 5, h, W), _cfg(k, base, 1))
    np.savez(f"{out}.{rank}.npz", logits=step.last_logits.cpu().numpy(), loss=float(loss),
             conf=conf.cpu().numpy(), **mk,
             **{"g_" + kk: p.grad.cpu().numpy() for kk, p in core.named_parameters(remove_duplicate=False)
                if p.grad is not None})
    dist.barrier()
    dist.destroy_process_group()


def _worker(rank, world, port, math_mode, out, depth):
    import pathlib
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests"), str(root / "spff-unet-spcct_amd")]
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
    mk = _save_masks(core, (SHAPE[0], SHAPE[1], d, SHAPE[3], SHAPE[4]), _cfg())
    np.savez(f"{out}.{rank}.npz", logits=step.last_logits.cpu().numpy(), loss=float(loss),
             conf=conf.cpu().numpy(), **mk,
             **{"g_" + k: p.grad.cpu().numpy() for k, p in core.named_parameters(remove_duplicate=False)
                if p.grad is not None})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,math_mode,depth", [
    (2, "f32", 8), (4, "f32", 8), (2, "bf16x6", 8), (4, "bf16x6", 8), (2, "bf16x6", 16),
    (2, "f16x3", 8)])
def test_depth_sharded_engine_matches_unsharded(tmp_path, world, math_mode, depth):
    import innovative3D.helpers as Hh
    core = _model(math_mode, depth)
    st = core._synth_state
    x, y = _data(depth)
    logits = core(x.cuda())
    loss, conf = Hh.ce_dice_with_confusion(logits, y.cuda(), K, 255)
    loss.backward()
    ref = logits.detach().cpu().numpy()
    grads = {k: p.grad.cpu().numpy() for k, p in core.named_parameters(remove_duplicate=False) if p.grad is not None}
    out = str(tmp_path / "sh")
    mp.spawn(_worker, args=(world, _free_port(), math_mode, out, depth), nprocs=world, join=True)
    parts = [np.load(f"{out}.{r}.npz") for r in range(world)]
    lg = np.concatenate([p["logits"] for p in parts], axis=2)
    e = float(np.abs(lg - ref).max())
    print(f"world {world} {math_mode} D {depth}: max|dlogit| {e:.2e}, loss {float(parts[0]['loss']):.7f} "
          f"vs {float(loss):.7f}")
    assert e <= 1e-4 * float(np.abs(ref).max())
    assert abs(float(parts[0]["loss"]) - float(loss)) <= 1e-5 * abs(float(loss))
    nflip = int((lg.argmax(1) != ref.argmax(1)).sum())
    assert int(np.abs(parts[0]["conf"] - conf.cpu().numpy()).sum()) <= 2 * nflip
    for k in grads:
        for p in parts[1:]:
            np.testing.assert_array_equal(p["g_" + k], parts[0]["g_" + k])
    _check_vs_oracle(parts, 2, st, _cfg(), x, y, math_mode)


@pytest.mark.parametrize("world,math_mode,case,memory", [
    (2, "f32", "small", None), (4, "f32", "small", None), (2, "bf16x6", "small", None),
    (4, "bf16x6", "small", None), (2, "f16x3", "small", None),
    # the lean saved-activation layout (recomputed block outputs / decoder inputs)
    (2, "bf16x6", "small", "lean")])
def test_height_sharded_engine_matches_unsharded(tmp_path, world, math_mode, case, memory):
    import innovative3D.helpers as Hh
    B, H, W, k, base = HCASES[case]
    core = _model(math_mode, 5, k, base, 1)
    st = core._synth_state
    x, y = _hdata(case)
    logits = core(x.cuda())
    loss, conf = Hh.ce_dice_with_confusion(logits, y.cuda(), k, 255)
    loss.backward()
    ref = logits.detach().cpu().numpy()            # [B, K, D, H, W]
    grads = {kk: p.grad.cpu().numpy() for kk, p in core.named_parameters(remove_duplicate=False) if p.grad is not None}
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
    for kk in grads:
        for p in parts[1:]:
            np.testing.assert_array_equal(p["g_" + kk], parts[0]["g_" + kk])
    _check_vs_oracle(parts, 3, st, _cfg(k, base, 1), x, y, math_mode)


# ---- BASELINE config 4's split: 8 ranks, f16x3, >= 12 slices per rank
# 1 x 5 x 96 x 128^2, K = 13, base 32: each rank owns 12 depth slices, so the 32-wide
# level-0 f16x3 tiles (4 deep) give 3 depth tiles per rank and the convs take the
# overlapped path (engine.hip conv_halo: the interior tile while the halo is exchanged on
# the side stream, dpart 1, then the boundary tiles, dpart 2, each with its own per-launch
# operand maxima); the first, the last and six interior ranks all run.
W8_SHAPE, W8_K, W8_BASE = (1, 5, 96, 128, 128), 13, 32


def _w8_data():
    from innovative3D.synthetic import synthetic_batch
    return synthetic_batch(*W8_SHAPE, num_classes=W8_K, ignore_frac=0.02, seed=17)


def _w8_worker(rank, world, port, math_mode, out):
    import pathlib
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests"), str(root / "spff-unet-spcct_amd")]
    from innovative3D.sharded import DepthShardedSPFF, shard_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    B, C, D, H, W = W8_SHAPE
    core = _model(math_mode, D, W8_K, W8_BASE, C)
    x, y = _w8_data()
    off, d = shard_bounds(D, world, rank)
    step = DepthShardedSPFF(core, W8_K, 255)
    loss, conf = step.step(x[:, :, off:off + d].contiguous().cuda(), y[:, off:off + d].contiguous().cuda())
    torch.cuda.synchronize()
    mk = _save_masks(core, (B, C, d, H, W), _cfg(W8_K, W8_BASE, C))
    np.savez(f"{out}.{rank}.npz", logits=step.last_logits.cpu().numpy(), loss=float(loss),
             conf=conf.cpu().numpy(), launched=np.array(step.bucketer.launched), **mk,
             **{"g_" + k: p.grad.cpu().numpy() for k, p in core.named_parameters(remove_duplicate=False)
                if p.grad is not None})
    del step, core
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(900)
def test_depth_sharded_world8_f16x3_overlapped(tmp_path):
    import innovative3D.helpers as Hh
    from innovative3D.sharded import shard_bounds
    world, mth = 8, "f16x3"
    B, C, D, H, W = W8_SHAPE
    assert shard_bounds(D, world, 0)[1] >= 12
    core = _model(mth, D, W8_K, W8_BASE, C)
    st = core._synth_state
    x, y = _w8_data()
    logits = core(x.cuda())
    loss, conf = Hh.ce_dice_with_confusion(logits, y.cuda(), W8_K, 255)
    loss.backward()
    ref = logits.detach().cpu().numpy()
    loss_ref, conf_ref = float(loss), conf.cpu().numpy()
    nflat = sum(p.numel() for p in core.parameters() if p.grad is not None)
    del core, logits, loss
    torch.cuda.empty_cache()
    out = str(tmp_path / "w8")
    mp.spawn(_w8_worker, args=(world, _free_port(), mth, out), nprocs=world, join=True)
    parts = [np.load(f"{out}.{r}.npz") for r in range(world)]
    lg = np.concatenate([p["logits"] for p in parts], axis=2)
    e = float(np.abs(lg - ref).max())
    nflip = int((lg.argmax(1) != ref.argmax(1)).sum())
    spans = sorted(map(tuple, parts[0]["launched"]))
    print(f"world 8 {mth} 1x5x96x128^2: max|dlogit| {e:.2e} (max|logit| {np.abs(ref).max():.2f}), "
          f"argmax flips {nflip}, loss {float(parts[0]['loss']):.7f} vs {loss_ref:.7f}, "
          f"{len(spans)} bucketed gradient all-reduces")
    assert e <= 1e-4 * float(np.abs(ref).max())
    assert abs(float(parts[0]["loss"]) - loss_ref) <= 1e-5 * abs(loss_ref)
    assert int(np.abs(parts[0]["conf"] - conf_ref).sum()) <= 2 * nflip
    # the gradient went through the bucketer during the backward, every float once
    assert spans[0][0] == 0 and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert spans[-1][1] == nflat and len(spans) > 1
    for k in (f for f in parts[0].files if f.startswith("g_")):
        for p in parts[1:]:
            np.testing.assert_array_equal(p[k], parts[0][k])
    _check_vs_oracle(parts, 2, st, _cfg(W8_K, W8_BASE, C), x, y, mth, device="cuda")


# ---- RCCL on >= 2 GPUs: device halos + the bucketed gradient all-reduces
# interleaved with them (SPFF_SHARD_OVERLAP=1), one GPU per rank.  The driver's GPU test box
# has one GPU, where this skips; on a multi-GPU node it is the sharded RCCL path's check.
def _rccl_worker(rank, world, port, out, overlap):
    import pathlib
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests"), str(root / "spff-unet-spcct_amd")]
    os.environ["SPFF_SHARD_OVERLAP"] = "1" if overlap else "0"
    from innovative3D.sharded import DepthShardedSPFF, shard_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", rank)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    depth = 16
    core = _model("f16x3", depth).to(dev)
    x, y = _data(depth)
    off, d = shard_bounds(depth, world, rank)
    step = DepthShardedSPFF(core, K, 255)
    assert (step.bucketer is not None) == overlap
    loss, conf = step.step(x[:, :, off:off + d].contiguous().to(dev),
                           y[:, off:off + d].contiguous().to(dev))
    torch.cuda.synchronize()
    mk = _save_masks(core, (SHAPE[0], SHAPE[1], d, SHAPE[3], SHAPE[4]), _cfg())
    np.savez(f"{out}.{rank}.npz", logits=step.last_logits.cpu().numpy(), loss=float(loss),
             conf=conf.cpu().numpy(), **mk,
             **{"g_" + k: p.grad.cpu().numpy() for k, p in core.named_parameters(remove_duplicate=False)
                if p.grad is not None})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs (one rank per GPU, RCCL)")
@pytest.mark.parametrize("overlap", [True, False])
def test_depth_sharded_rccl_two_gpus(tmp_path, overlap):
    import innovative3D.helpers as Hh
    depth = 16
    core = _model("f16x3", depth)
    st = core._synth_state
    x, y = _data(depth)
    logits = core(x.cuda())
    loss, _conf = Hh.ce_dice_with_confusion(logits, y.cuda(), K, 255)
    loss.backward()
    ref, loss_ref = logits.detach().cpu().numpy(), float(loss)
    del core, logits, loss
    out = str(tmp_path / "rccl")
    mp.spawn(_rccl_worker, args=(2, _free_port(), out, overlap), nprocs=2, join=True)
    parts = [np.load(f"{out}.{r}.npz") for r in range(2)]
    lg = np.concatenate([p["logits"] for p in parts], axis=2)
    e = float(np.abs(lg - ref).max())
    print(f"RCCL world 2 overlap={overlap}: max|dlogit| {e:.2e}, loss {float(parts[0]['loss']):.7f} "
          f"vs {loss_ref:.7f}")
    assert e <= 1e-4 * float(np.abs(ref).max())
    assert abs(float(parts[0]["loss"]) - loss_ref) <= 1e-5 * abs(loss_ref)
    for k in (f for f in parts[0].files if f.startswith("g_")):
        np.testing.assert_array_equal(parts[1][k], parts[0][k])
    _check_vs_oracle(parts, 2, st, _cfg(), x, y, "f16x3")
