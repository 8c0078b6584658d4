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
