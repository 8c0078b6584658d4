"""BASELINE configs[3] at its own size: ONE 1 x 5 x 512^3 volume (K = 13, base 32, f16x3),
depth-sharded into 8 slabs of 64 slices (the north star's 8-GPU split: first, last and
six interior ranks), against the SAME volume run whole on one GPU (lean layout, 211 GiB).

The box has one GPU, and RCCL refuses two ranks on one device, so the 8 ranks share it
through host-staged gloo (innovative3D.sharded.TorchDepthColl) -- the same spff_coll
callbacks and engine code paths as the RCCL run, including the overlapped halo of the
depth-sharded convs.  The 1-GPU run goes first in this process (its logits kept in host
memory, its 211 GiB workspace released before the ranks start); each rank then runs its
slab (a ~28 GiB lean plan) and writes its logits slab to /dev/shm.

Size-independent properties (no CPU oracle at 134 M voxels): gathered logits within
1e-4 of max|logit| of the 1-GPU logits, loss within 1e-5 relative, argmax flips only at
near-ties (top-2 margin of the 1-GPU logits < 2 max|dlogit|), every rank holding the
same all-reduced gradient, and the gradient's relative L2 distance to the 1-GPU one
printed per tensor (two fp32 sums over 134 M voxels in different orders, with
LeakyReLU / max-pool knife edges; reported, bounded loosely).  Marked gpu."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
SHAPE, K, BASE, WORLD = (1, 5, 512, 512, 512), 13, 32, 8
SHM = "/dev/shm"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(D):
    import innovative3D.models as M
    from innovative3D.weightgen import synth_state
    core = M.build_spct_energyfilm_fourier(num_classes=K, base=BASE, in_channels=SHAPE[1])
    for b in core._blocks():
        b.fgate._ensure_mask(D, "cpu")
    st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=0)
    core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    core = core.to("cuda")
    core.math = "f16x3"
    core.memory = "lean"
    return core


def _worker(rank, world, port, tag):
    import pathlib
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests"), str(root / "spff-unet-spcct_amd")]
    from innovative3D.sharded import DepthShardedSPFF, shard_bounds
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import datetime
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=900))
    torch.cuda.set_device(0)
    D = SHAPE[2]
    off, d = shard_bounds(D, world, rank)
    x = np.load(f"{SHM}/{tag}_x.npy", mmap_mode="r")
    y = np.load(f"{SHM}/{tag}_y.npy", mmap_mode="r")
    xs = torch.from_numpy(np.ascontiguousarray(x[:, :, off:off + d])).cuda()
    ys = torch.from_numpy(np.ascontiguousarray(y[:, off:off + d])).cuda()
    core = _model(D)
    step = DepthShardedSPFF(core, K, 255, timeout=900.0)
    loss, _conf = step.step(xs, ys)
    torch.cuda.synchronize()
    np.save(f"{SHM}/{tag}_lg{rank}.npy", step.last_logits.cpu().numpy())
    g = {k: p.grad.detach().cpu().numpy() for k, p in core.named_parameters(remove_duplicate=False)
         if p.grad is not None and not k.endswith("._mask")}
    np.savez(f"{SHM}/{tag}_g{rank}.npz", loss=float(loss), **g)
    del step, core, xs, ys
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(1500)
def test_volume512_depth_sharded_8_ranks_matches_one_gpu():
    import innovative3D._engine as E
    import innovative3D.helpers as Hh
    from innovative3D.synthetic import synthetic_batch
    tag = f"spff_v512_{os.getpid()}"
    files = []
    try:
        x, y = synthetic_batch(*SHAPE, num_classes=K, ignore_frac=0.01, seed=1000)
        for nm, a in (("x", x), ("y", y)):
            np.save(f"{SHM}/{tag}_{nm}.npy", a.numpy())
            files.append(f"{SHM}/{tag}_{nm}.npy")
        # --- the whole volume on one GPU (lean layout) ---
        core = _model(SHAPE[2])
        logits = core(x.cuda())
        loss, _conf = Hh.ce_dice_with_confusion(logits, y.cuda(), K, 255)
        loss.backward()
        torch.cuda.synchronize()
        ref = logits.detach().cpu().numpy()          # [1, K, D, H, W] (7 GB)
        loss1 = float(loss)
        g1 = {k: p.grad.detach().cpu().numpy() for k, p in core.named_parameters(remove_duplicate=False)
              if p.grad is not None and not k.endswith("._mask")}
        del core, logits, loss, x, y
        E.release_plans()
        torch.cuda.empty_cache()
        # --- 8 depth slabs of 64 slices, one process each, host-staged gloo ---
        mp.spawn(_worker, args=(WORLD, _free_port(), tag), nprocs=WORLD, join=True)
        files += [f"{SHM}/{tag}_lg{r}.npy" for r in range(WORLD)]
        files += [f"{SHM}/{tag}_g{r}.npz" for r in range(WORLD)]
        amax = float(np.abs(ref).max())
        d = SHAPE[2] // WORLD
        err, nflip, nflip_tie = 0.0, 0, 0
        for r in range(WORLD):
            lg = np.load(f"{SHM}/{tag}_lg{r}.npy")
            rs = ref[:, :, r * d:(r + 1) * d]
            e = float(np.abs(lg - rs).max())
            err = max(err, e)
            fl = lg.argmax(1) != rs.argmax(1)
            top2 = np.sort(rs, axis=1)[:, -2:]
            nflip += int(fl.sum())
            nflip_tie += int((fl & ((top2[:, 1] - top2[:, 0]) < 2 * e)).sum())
            del lg
        parts = [np.load(f"{SHM}/{tag}_g{r}.npz") for r in range(WORLD)]
        loss8 = float(parts[0]["loss"])
        print(f"volume 1x5x512^3, 8 depth slabs vs 1 GPU: max|dlogit| {err:.2e} (max|logit| "
              f"{amax:.2f}), argmax flips {nflip} of {ref[:, 0].size} ({nflip_tie} at near-ties), "
              f"loss {loss8:.8f} vs {loss1:.8f}")
        rows = []
        for k, g in g1.items():
            a = parts[0][k].astype(np.float64).reshape(-1)
            b = g.astype(np.float64).reshape(-1)
            rows.append((float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)), k))
            for p in parts[1:]:
                np.testing.assert_array_equal(p[k], parts[0][k])
        rows.sort(reverse=True)
        for rel, k in rows[:6]:
            print(f"  grad {k:34s} rel L2 vs 1 GPU {rel:.2e}")
        assert err <= 1e-4 * amax
        assert abs(loss8 - loss1) <= 1e-5 * abs(loss1)
        assert nflip == nflip_tie, f"{nflip - nflip_tie} argmax flips outside near-ties"
        # two fp32 sums over 134 M voxels in different orders, plus the knife-edge branches
        # each run takes on its own (no oracle to force them at this size): observed 3.6e-3
        assert rows[0][0] <= 1e-2, rows[:3]
    finally:
        for f in files:
            try:
                os.remove(f)
            except OSError:
                pass
