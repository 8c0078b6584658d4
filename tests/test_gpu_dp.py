"""Batch data parallelism through the engine (innovative3D.distributed.DataParallelSPFF)
on ONE GPU: 2 ranks, each its own process, plan and sample, gloo on device
tensors.  Exercises the engine's gradient-ready hook (spff_plan_set_grad_hook):
the bucketed all-reduces are issued DURING the backward and must cover every
gradient float once.  The all-reduced gradients, the global loss and the global
confusion must equal the single-process engine on the concatenated batch
(SURVEY §8(e) DP row; helpers.py:782-803).  Marked gpu."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
K, BASE, SHAPE = 7, 8, (2, 5, 8, 32, 32)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    import innovative3D.models as M
    from innovative3D.weightgen import synth_state
    lit = M.LitSPCT_EFiLM_FourierGate(num_classes=K, base=BASE)
    # the registry module is Cin=1; the north-star layout takes 5 channels
    core = M.build_spct_energyfilm_fourier(num_classes=K, base=BASE, in_channels=SHAPE[1])
    lit.model = core
    for b in core._blocks():
        b.fgate._ensure_mask(SHAPE[2], "cpu")
    st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=9,
                     mask_jitter=0.25)
    core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    return lit.to("cuda")


def _data():
    from innovative3D.synthetic import synthetic_batch
    return synthetic_batch(*SHAPE, num_classes=K, ignore_frac=0.05, seed=21)


def _worker(rank, world, port, bucket, out):
    import pathlib
    import sys
    root = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(root), str(root / "spff-unet-spcct_amd")]
    from innovative3D.distributed import DataParallelSPFF
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    lit = _model()
    x, y = _data()
    dp = DataParallelSPFF(lit, K, 255, bucket_bytes=bucket)
    loss, conf = dp.step(x[rank:rank + 1].cuda(), y[rank:rank + 1].cuda())
    torch.cuda.synchronize()
    launched = list(dp.bucketer.launched)
    np.savez(f"{out}.{rank}.npz", loss=float(loss), conf=conf.cpu().numpy(),
             launched=np.array(launched),
             **{"g_" + k: p.grad.cpu().numpy() for k, p in lit.named_parameters()
                if p.grad is not None})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket", [1 << 14, 1 << 30])
def test_dp_engine_matches_full_batch(tmp_path, bucket):
    import innovative3D.helpers as Hh
    lit = _model()
    x, y = _data()
    logits = lit(x.cuda())
    loss, conf = Hh.ce_dice_with_confusion(logits, y.cuda(), K, 255)
    loss.backward()
    grads = {k: p.grad.cpu().numpy() for k, p in lit.named_parameters() if p.grad is not None}
    out = str(tmp_path / "dp")
    mp.spawn(_worker, args=(2, _free_port(), bucket, out), nprocs=2, join=True)
    parts = [np.load(f"{out}.{r}.npz") for r in range(2)]
    spans = sorted(map(tuple, parts[0]["launched"]))
    print(f"bucket {bucket} B: {len(spans)} all-reduces, loss {float(parts[0]['loss']):.8f} vs "
          f"{float(loss):.8f}")
    assert spans[0][0] == 0 and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert spans[-1][1] == sum(int(np.prod(g.shape)) for g in grads.values())
    if bucket < (1 << 20):
        assert len(spans) > 3  # several buckets issued while the backward ran
    for p in parts:
        assert abs(float(p["loss"]) - float(loss)) <= 2e-7 * abs(float(loss))
        np.testing.assert_array_equal(p["conf"], conf.cpu().numpy())
    for k, g in grads.items():
        sc = max(float(np.abs(g).max()), 1e-30)
        e = float(np.abs(parts[0]["g_" + k] - g).max()) / sc
        assert e <= 1e-4, (k, e)
        np.testing.assert_array_equal(parts[1]["g_" + k], parts[0]["g_" + k])


@pytest.mark.timeout(300)
def test_rccl_world1_bucketed_step(tmp_path):
    """The RCCL device path on the box's one GPU: a world-1 "nccl" process group
    (RCCL on ROCm), one DataParallelSPFF step with every collective forced on -- the
    valid-count all-reduce, the bucketed gradient all-reduces issued from the engine's
    grad hook WHILE its backward is enqueued, the fp64 loss/confusion all-reduce -- and
    TorchDepthColl's device branches (all_reduce on the engine's side stream; a halo
    with no neighbour).  A SUM over one rank is the identity, so the gradients and the
    confusion must equal the step without a process group BITWISE (the loss to 2e-7).  Two ranks on one
    GPU are refused by RCCL (ncclInvalidUsage: Duplicate GPU), so the sharded halo's
    device exchange between peers needs >= 2 GPUs."""
    import innovative3D.helpers as Hh
    from innovative3D.distributed import DataParallelSPFF
    from innovative3D.sharded import TorchDepthColl
    assert not dist.is_initialized()
    torch.cuda.set_device(0)
    lit = _model()
    x, y = _data()
    x, y = x[:1].cuda(), y[:1].cuda()
    logits = lit(x)
    loss0, conf0 = Hh.ce_dice_with_confusion(logits, y, K, 255)
    loss0.backward()
    torch.cuda.synchronize()
    ref = {k: p.grad.clone() for k, p in lit.named_parameters() if p.grad is not None}
    nflat = sum(g.numel() for g in ref.values())
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}",
                            rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        backend = dist.get_backend()
        print(f"backend {backend}, world {dist.get_world_size()}")
        assert backend == "nccl"
        dp = DataParallelSPFF(lit, K, 255, bucket_bytes=1 << 14, force_collectives=True)
        loss, conf = dp.step(x, y)
        torch.cuda.synchronize()
        spans = sorted(dp.bucketer.launched)
        print(f"{len(spans)} bucketed RCCL all-reduces; loss {float(loss):.8f} vs {float(loss0):.8f}")
        assert dp.bucketer.begun == 1 and len(spans) > 3
        assert spans[0][0] == 0 and all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert spans[-1][1] == nflat
        # the global loss is re-formed from the all-reduced fp64 [CE, confusion] buffer
        # (distributed.global_loss): equal to the last fp32 bit or one ulp
        assert abs(float(loss) - float(loss0)) <= 2e-7 * abs(float(loss0))
        assert torch.equal(conf.cpu(), conf0.cpu().to(conf.dtype))
        for k, p in lit.named_parameters():
            if p.grad is not None:
                assert torch.equal(p.grad, ref[k]), k
        # TorchDepthColl's device branches, on a side stream as the engine hands them
        coll = TorchDepthColl()
        assert not coll.host
        s2 = torch.cuda.Stream()
        t = torch.randn(1000, dtype=torch.float64, device="cuda")
        slab = torch.randn(6 * 64, device="cuda")
        t0, slab0 = t.clone(), slab.clone()
        s2.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s2):
            coll.allreduce(t)
            coll.halo(slab, 64, 4)
        torch.cuda.synchronize()
        assert torch.equal(t, t0) and torch.equal(slab, slab0)
    finally:
        dist.destroy_process_group()
