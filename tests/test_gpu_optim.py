"""Fused Adam / AdamW (innovative3D.optim.SPFFAdam, include/spff.h spff_adam_step)
against torch.optim.Adam / AdamW on the GPU: flat-buffer parameters (the
engine's layout) and separately allocated ones, with and without weight decay,
several steps; then a real SPFF-UNet training step.  Marked gpu."""
import pytest
import torch

from innovative3D.optim import SPFFAdam

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(flat, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(32, 16, 3, 3, 3), (32,), (7, 5), (1,), (257,)]
    n = sum(torch.Size(s).numel() for s in shapes)
    if flat:
        buf = torch.randn(n, generator=g).to(DEV)
        gbuf = torch.empty(n, device=DEV)
        ps, o = [], 0
        for s in shapes:
            k = torch.Size(s).numel()
            p = torch.nn.Parameter(buf[o:o + k].view(s))
            p.grad = gbuf[o:o + k].view(s)
            ps.append(p)
            o += k
        return ps
    return [torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for s in shapes]


@pytest.mark.parametrize("flat", [True, False])
@pytest.mark.parametrize("wd,decoupled", [(0.0, False), (1e-2, False), (1e-2, True)])
def test_fused_adam_matches_torch(flat, wd, decoupled):
    a = _params(flat)
    b = [torch.nn.Parameter(p.detach().clone()) for p in a]
    ref = (torch.optim.AdamW if decoupled else torch.optim.Adam)(b, lr=3e-3, weight_decay=wd)
    opt = SPFFAdam(a, lr=3e-3, weight_decay=wd, decoupled_weight_decay=decoupled)
    g = torch.Generator().manual_seed(1)
    worst = 0.0
    for _ in range(5):
        for pa, pb in zip(a, b):
            gr = torch.randn(pa.shape, generator=g).to(DEV)
            if pa.grad is None:
                pa.grad = gr.clone()
            else:
                pa.grad.copy_(gr)
            pb.grad = gr.clone()
        opt.step()
        ref.step()
        for pa, pb in zip(a, b):
            worst = max(worst, float((pa - pb).abs().max() / pb.abs().max()))
    print(f"flat={flat} wd={wd} decoupled={decoupled}: max rel diff {worst:.2e}")
    assert worst <= 1e-6
    # the state layout is torch's
    st = opt.state_dict()["state"][0]
    assert set(st) >= {"step", "exp_avg", "exp_avg_sq"} and int(st["step"]) == 5


def test_fused_adam_on_spff_training_step():
    import innovative3D.models as M
    from innovative3D.weightgen import synth_state
    from innovative3D.helpers import ce_plus_macro_dice_loss
    from innovative3D.synthetic import synthetic_batch
    x, y = synthetic_batch(1, 5, 8, 32, 32, num_classes=5, seed=3, device=DEV)

    def make():
        core = M.build_spct_energyfilm_fourier(num_classes=5, base=8, in_channels=5)
        st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=2)
        core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
        return core.to(DEV)
    a, b = make(), make()
    oa = SPFFAdam(a.parameters(), lr=1e-3)            # built before the first forward: the
    ob = torch.optim.Adam(b.parameters(), lr=1e-3)    # lazy FourierGate masks are not in it
    pa = dict(a.named_parameters())
    pb = dict(b.named_parameters())
    for _ in range(3):
        # the engine's gradients of model a (flat-buffer layout) drive both optimizers, so
        # the comparison is of the optimizers, not of two diverging trajectories
        oa.zero_grad(set_to_none=True)
        ce_plus_macro_dice_loss(a(x), y, 5).backward()
        for k, p in pb.items():
            p.grad = None if pa[k].grad is None else pa[k].grad.detach().clone()
        oa.step()
        ob.step()
        worst = max(float((pa[k] - pb[k]).abs().max() / max(float(pb[k].abs().max()), 1e-12))
                    for k in pb)
        assert worst <= 1e-6, worst
    # the FourierGate masks, created lazily by the first forward (after the optimizer),
    # are not optimised: still the ones they were created as
    assert torch.all(a.state_dict()["enc1.fgate.freq_mask"] == 1)
