"""SPFF_MEM_LEAN layout (include/spff.h memory_mode): the backward recomputes the
block activations, the decoder inputs and the up-conv outputs it no longer
saves.  Same kernels, same operands -> the lean engine must be BITWISE equal
to the full-save engine (logits, loss, every gradient), unsharded and
depth-sharded (world 2 on one GPU, host-staged gloo).  Marked gpu."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
K, BASE, SHAPE = 6, 8, (2, 5, 8, 32, 32)


def _model(math_mode, memory, shape=SHAPE):
    import innovative3D.models as M
    from innovative3D.weightgen import synth_state
    core = M.build_spct_energyfilm_fourier(num_classes=K, base=BASE, in_channels=shape[1])
    for b in core._blocks():
        b.fgate._ensure_mask(shape[2], "cpu")
    st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=13,
                     mask_jitter=0.25)
    core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    core = core.to("cuda")
    core.math, core.memory = math_mode, memory
    return core


def _run(core, x, y):
    import innovative3D.helpers as Hh
    logits = core(x.cuda())
    loss, conf = Hh.ce_dice_with_confusion(logits, y.cuda(), K, 255)
    loss.backward()
    torch.cuda.synchronize()
    return (logits.detach().cpu(), float(loss), conf.cpu(),
            {k: p.grad.cpu() for k, p in core.named_parameters(remove_duplicate=False)})


@pytest.mark.parametrize("math_mode", ["f32", "bf16x6", "f16x3"])
def test_lean_equals_full_bitwise(math_mode):
    from innovative3D.synthetic import synthetic_batch
    x, y = synthetic_batch(*SHAPE, num_classes=K, ignore_frac=0.05, seed=3)
    full = _model(math_mode, "full")
    lean = _model(math_mode, "lean")
    rf, rl = _run(full, x, y), _run(lean, x, y)
    assert full._plan.memory == "full" and lean._plan.memory == "lean"
    # at 40K voxels the size-independent part (packed weights, stats) is a large share;
    # the per-voxel ratio at production sizes is asserted in tests/test_abi_cpu.py
    assert lean._plan.ws_bytes < 0.75 * full._plan.ws_bytes
    assert torch.equal(rf[0], rl[0])
    assert rf[1] == rl[1]
    assert torch.equal(rf[2], rl[2])
    for k, g in rf[3].items():
        assert torch.equal(g, rl[3][k]), k
    # a second step on the same plans (workspace reuse) stays identical
    for m in (full, lean):
        for p in m.parameters():
            p.grad = None
    r2 = _run(lean, x, y)
    for k, g in rf[3].items():
        assert torch.equal(g, r2[3][k]), k


def test_lean_equals_full_ragged_hw():
    """H, W not multiples of 8 (36 x 44: the _cat trilinear resize at level 2 in H and
    W): the lean layout recomputes the up-conv output through the same resize."""
    from innovative3D.synthetic import synthetic_batch
    shp = (1, 5, 8, 36, 44)
    x, y = synthetic_batch(*shp, num_classes=K, ignore_frac=0.05, seed=4)
    rf = _run(_model("bf16x6", "full", shp), x, y)
    rl = _run(_model("bf16x6", "lean", shp), x, y)
    assert torch.equal(rf[0], rl[0])
    assert rf[1] == rl[1]
    for k, g in rf[3].items():
        assert torch.equal(g, rl[3][k]), k


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SH = (1, 5, 8, 32, 32)


def _worker(rank, world, port, out, memory="lean"):
    import pathlib
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "tests"), str(root / "spff-unet-spcct_amd")]
    from test_gpu_memory import SH, _model
    from innovative3D.sharded import DepthShardedSPFF, shard_bounds
    from innovative3D.synthetic import synthetic_batch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    core = _model("bf16x6", memory, SH)
    x, y = synthetic_batch(*SH, num_classes=K, ignore_frac=0.05, seed=8)
    off, d = shard_bounds(SH[2], world, rank)
    step = DepthShardedSPFF(core, K, 255)
    loss, conf = step.step(x[:, :, off:off + d].contiguous().cuda(), y[:, off:off + d].contiguous().cuda())
    torch.cuda.synchronize()
    np.savez(f"{out}.{rank}.npz", logits=step.last_logits.cpu().numpy(), loss=float(loss),
             lean=int(core._plan.memory == "lean"), full=int(core._plan.memory == "full"),
             **{"g_" + k: p.grad.cpu().numpy() for k, p in core.named_parameters()
                if p.grad is not None})
    dist.barrier()
    dist.destroy_process_group()


def test_lean_sharded_matches_full_sharded(tmp_path):
    """world-2 depth-sharded, lean layout vs the same volume sharded under the full
    layout: same kernels, same operands -> bitwise equal (tests/test_gpu_sharded.py
    pins the full sharded engine to the unsharded one)."""
    res = {}
    for mem in ("full", "lean"):
        out = str(tmp_path / mem)
        mp.spawn(_worker, args=(2, _free_port(), out, mem), nprocs=2, join=True)
        res[mem] = [np.load(f"{out}.{r}.npz") for r in range(2)]
    assert all(int(p["lean"]) for p in res["lean"]) and all(int(p["full"]) for p in res["full"])
    for r in range(2):
        a, b = res["full"][r], res["lean"][r]
        assert np.array_equal(a["logits"], b["logits"]), r
        assert float(a["loss"]) == float(b["loss"])
        for k in a.files:
            if k.startswith("g_"):
                assert np.array_equal(a[k], b[k]), (r, k)
