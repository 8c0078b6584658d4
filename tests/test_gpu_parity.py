"""Whole-network parity of the HIP engine against the golden fixtures produced
by the reference itself (tests/golden/make_golden.py), plus stage-wise
localisation against the CPU oracle.  Marked gpu.

Tolerances (north star, BASELINE.json): logits within 1e-3 of the reference
PyTorch-CPU forward, identical argmax (voxels whose reference top-2 margin is
below 2 x the observed max |dlogit| are reported as near-ties, not failures);
gradients vs a kink-consistent fp64 oracle (engine_lrelu_masks) within
max(1e-3, 8 x the fp32 oracle's own error) of max|g| per tensor (some
gate-parameter gradients are cancelling sums the fp32 reference itself only
gets to ~5e-2; FourierGate mag_scale, whose gradient sum_k mask_k dL/dM_k cancels
almost completely, is judged against the sum of its absolute terms); loss within
1e-5 relative.  Max-pool windows route the oracle's gradient through the
engine's own argmax, like the LeakyReLU signs."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from _golden import cfg_of, fixture_names, load, state_of
from _golden import build_core as _build_core
from oracle import spff_oracle as O
import innovative3D.models as M
import innovative3D.helpers as Hh

pytestmark = pytest.mark.gpu
DEV = "cuda"


def build_core(meta):
    return _build_core(meta)


def load_core(d):
    meta = d["meta"]
    core = build_core(meta)
    D = d["x"].shape[2]
    for b in core._blocks():
        if isinstance(getattr(b, "fgate", None), M.FourierGate3D):
            b.fgate._ensure_mask(D, "cpu")
    st = state_of(d)
    core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()}, strict=True)
    return core.to(DEV)


def near_tie_mask(ref_logits, tol):
    top2 = np.sort(ref_logits, axis=1)[:, -2:]
    return (top2[:, 1] - top2[:, 0]) < tol


@pytest.mark.parametrize("mth", ["f32", "bf16x6", "bf16x3", "f16x3"])
@pytest.mark.parametrize("name", fixture_names())
def test_network_matches_reference(name, mth):
    """f32, bf16x6 (the fp32-faithful split) and f16x3 (scaled fp16 planes) are held to
    the same bar;
    bf16x3 (opt-in, ~2^-17 per product) to the same logits / argmax bar, loss
    within 1e-4 and gradients within max(5e-3, 64 x the fp32 oracle's error)."""
    d = load(name)
    meta = d["meta"]
    K = meta["K"]
    core = load_core(d)
    core.math = mth
    x = torch.from_numpy(d["x"]).to(DEV)
    y = torch.from_numpy(d["labels"]).to(DEV)
    logits = core(x)
    loss, conf = Hh.ce_dice_with_confusion(logits, y, K, 255)
    loss.backward()
    torch.cuda.synchronize()
    lg = logits.detach().cpu().numpy()
    ref = d["logits"]
    err = float(np.abs(lg - ref).max())
    print(f"{name}/{mth}: max|dlogit| = {err:.3e}  loss {float(loss):.7f} vs {float(d['loss']):.7f}")
    assert err <= 1e-3
    am, am_ref = lg.argmax(1), ref.argmax(1)
    flips = am != am_ref
    if flips.any():
        ties = near_tie_mask(ref, 2 * err)
        assert not (flips & ~ties).any(), f"{int(flips.sum())} argmax flips outside near-ties"
    assert math.isclose(float(loss), float(d["loss"]), rel_tol=1e-4 if mth == "bf16x3" else 1e-5)
    met = M.metrics_from_confusion(conf.cpu().numpy(), K, int(y.numel()))
    if not flips.any():
        np.testing.assert_allclose(np.array(met[0]), d["met_dice"], rtol=1e-12, equal_nan=True)
        np.testing.assert_allclose(np.array(met[3:]), d["met_scalars"], rtol=1e-12, equal_nan=True)
    # gradients: vs a kink-consistent fp64 oracle (see oracle_grads), tolerance =
    # max(1e-3, 8 x the fp32 oracle's own error) of max|g| per tensor
    named = dict(core.named_parameters(remove_duplicate=False))
    masks = engine_lrelu_masks(core, d)
    ref64, ref32, nflip, absb = oracle_grads(d, masks)
    print(f"  LeakyReLU kink flips (engine vs fp64 sign): {nflip}")
    check_grads({k: named[k].grad for k in ref64}, ref64, ref32, absb, state_of(d), mth)


def check_grads(grads, ref64, ref32, absb, st, mth):
    """Every engine gradient vs the kink-consistent fp64 oracle: max|g - g64| / scale
    within max(1e-3, 8 x the fp32 oracle's own error) (bf16x3: max(5e-3, 64 x); the
    floor alone when ``ref32`` is None); scale
    = max over the tensor of sum_b |per-sample g_b| (absb); FourierGate mag_scale is
    judged against the sum of its absolute terms."""
    rows, bad = [], []
    for kk, g64 in ref64.items():
        g = grads[kk]
        assert g is not None, kk
        g = np.asarray(g.detach().double().cpu().numpy() if torch.is_tensor(g) else g, np.float64)
        # scale: sum over samples of |per-sample gradient| (= max|g| for B=1); the batch
        # gradient is a sum of per-sample terms that can cancel (e.g. SE biases)
        scale = max(float(absb[kk].max()), 1e-12)
        if kk.endswith("fgate.mag_scale"):
            # d/d(mag) = sum_k mask_k dL/dM_k (M = mask * mag): a sum over the rfft
            # bins that can cancel almost completely; judge it against the sum of
            # its absolute terms, sum_k |mask_k dL/dM_k| = sum_k |mask_k g_mask_k| / |mag|
            pre = kk[: -len("mag_scale")]
            mk = pre + ("freq_mask" if pre + "freq_mask" in ref64 else "_mask")
            mag = abs(float(np.asarray(st[kk]).reshape(-1)[0]))
            terms = np.abs(np.asarray(st[pre + "freq_mask"]).reshape(-1) *
                           absb[mk].reshape(-1)).sum()
            scale = max(scale, float(terms) / max(mag, 1e-12))
        e_gpu = float(np.abs(g - g64).max()) / scale
        e_32 = float(np.abs(ref32[kk] - g64).max()) / scale if ref32 is not None else 0.0
        tol = max(5e-3, 64 * e_32) if mth == "bf16x3" else max(1e-3, 8 * e_32)
        rows.append((e_gpu, e_32, kk))
        if e_gpu > tol:
            bad.append(f"{kk}: gpu {e_gpu:.2e} vs fp32-oracle {e_32:.2e}")
    rows.sort(reverse=True)
    print("\n".join(f"  {k:32s} gpu {a:.2e}  fp32-oracle {b:.2e}" for a, b, k in rows[:6]))
    assert not bad, "; ".join(bad)


def _block_names(cfg):
    a, b = ("pre", "body") if cfg.novel else ("b1", "b2")
    return [(blk, a, b) for blk in ("enc1", "enc2", "enc3", "bott", "dec3", "dec2", "dec1")]


def engine_lrelu_masks(core, d):
    return engine_branch_masks(core, d["x"].shape, state_of(d), cfg_of(d["meta"]))


def engine_branch_masks(core, xshape, st, cfg):
    """Sign pattern of every LeakyReLU input, and the argmax of every max-pool
    window, as the ENGINE saw them (the pools: from its saved pool inputs; ties
    resolved first-max like the engine and torch).  The LeakyReLUs: the engine's
    saved conv outputs y1/y2 under its own per-(b,c) affine (al, de).  A fp32 conv differs from the
    reference's by ~1e-6 relative, so an input sitting within that of the kink
    (|r| ~ 0) can take the other slope (1 vs 0.01) -- a legitimate fp32 outcome
    the reference could equally produce.  Feeding the engine's pattern to the
    oracle removes these knife-edge flips from the gradient comparison."""
    B = xshape[0]
    plan = core._plan
    masks = {}
    for blk, a, b in _block_names(cfg):
        for tag, key in ((a, "y1"), (b, "y2")):
            y = plan.saved(f"{blk}.{key}").double().cpu()
            C = y.shape[1]
            Dd = xshape[2]
            lvl = {"enc1": 0, "dec1": 0, "enc2": 1, "dec2": 1, "enc3": 2, "dec3": 2, "bott": 3}[blk]
            Hh_, Ww = xshape[3] >> lvl, xshape[4] >> lvl
            y = y.view(B, Dd, Hh_, Ww, C).permute(0, 4, 1, 2, 3)
            g = torch.from_numpy(st[f"{blk}.{tag}.1.weight"]).double()
            bb = torch.from_numpy(st[f"{blk}.{tag}.1.bias"]).double()
            m64 = F.instance_norm(y, weight=g, bias=bb, eps=1e-5) > 0
            # the engine's own fp32 normalisation r = fma(y, al, de): its sign is the
            # sign of the exact y*al + de, which fp64 reproduces
            j = "1" if key == "y1" else "2"
            al = plan.saved(f"{blk}.al{j}").double().cpu().reshape(B, C, 1, 1, 1)
            de = plan.saved(f"{blk}.de{j}").double().cpu().reshape(B, C, 1, 1, 1)
            # contiguous: this torch build's CPU instance_norm backward is wrong for a
            # channels-last-strided grad_output, which torch.where would propagate
            m = ((y * al + de) > 0).contiguous()
            nd = int((m != m64).sum())
            if nd:
                print(f"  {blk}.{tag}: {nd} knife-edge signs (engine affine vs fp64 IN)")
            masks[f"{blk}.{tag}"] = m
    # max-pool windows: the engine's own argmax bytes (k = 2 dh + dw, first max in scan
    # order), as its backward routed them -- also valid for lean plans, whose block
    # outputs live in backward scratch
    Dd = xshape[2]
    for k in range(3):
        Hh_, Ww = xshape[3] >> (k + 1), xshape[4] >> (k + 1)
        idx = plan.saved(f"pool{k + 1}.idx").to(torch.int64).cpu()
        C = idx.shape[1]
        masks[f"pool{k + 1}"] = idx.view(B, Dd, Hh_, Ww, C).permute(0, 4, 1, 2, 3).contiguous()
    return masks


def oracle_grads(d, masks):
    return oracle_grads_st(cfg_of(d["meta"]), state_of(d), d["x"], d["labels"], masks)


def oracle_grads_st(cfg, st, x, labels, masks, device="cpu", fp32=True):
    """fp64 and fp32 oracle parameter gradients (CPU; ``device`` evaluates the same
    restatement through PyTorch's fp64 device kernels, ``fp32=False`` skips the fp32
    run and returns None for it) whose LeakyReLUs take the
    given sign patterns; also returns how many entries differ from the fp64
    oracle's own pattern (knife-edge flips) and sum_b |g_b| (fp64 per-sample
    gradients with the global CE normalisation; sum_b g_b = g exactly since
    IN / SE / gates are per sample and the Dice term carries no gradient).
    ``x``, ``labels``: numpy arrays; ``st``: the state dict (numpy)."""
    st = {k: v for k, v in st.items() if not k.endswith("._mask")}
    d = {"x": np.ascontiguousarray(x), "labels": np.ascontiguousarray(labels)}
    out = []
    nflip = [0]
    orig, orig_pool = O.conv_in_lrelu, O.maxpool
    npool = [0]
    masks = {k: v.to(device) for k, v in masks.items()}

    def pool_hooked(t):
        k = npool[0] % 3
        npool[0] += 1
        idx = masks[f"pool{k + 1}"]
        B_, C_, D_, H_, W_ = t.shape
        v = t[..., :H_ // 2 * 2, :W_ // 2 * 2].reshape(B_, C_, D_, H_ // 2, 2, W_ // 2, 2)
        v = v.permute(0, 1, 2, 3, 5, 4, 6)
        v = v.reshape(B_, C_, D_, H_ // 2, W_ // 2, 4)
        if t.dtype == torch.float64:
            nflip[0] += int((v.detach().argmax(-1) != idx).sum())
        return v.gather(-1, idx.unsqueeze(-1)).squeeze(-1)

    def hooked(P_, pre, inp, ksd):
        y = F.conv3d(inp, P_[pre + ".0.weight"], None, padding=(ksd // 2, 1, 1))
        r = F.instance_norm(y, weight=P_[pre + ".1.weight"], bias=P_[pre + ".1.bias"], eps=1e-5)
        m = masks[pre]
        if r.dtype == torch.float64:
            nflip[0] += int((m != (r.detach() > 0)).sum())
        return torch.where(m, r, 0.01 * r)

    O.conv_in_lrelu = hooked
    O.maxpool = pool_hooked
    try:
        for dt in ((torch.float64, torch.float32) if fp32 else (torch.float64,)):
            P = O.params_from_state(st, dtype=dt, device=device)
            O.fwd_bwd(P, torch.from_numpy(d["x"]).to(device, dt),
                      torch.from_numpy(d["labels"]).to(device), cfg)
            out.append({k: v.grad.double().cpu().numpy() for k, v in P.items()})
            del P
        if not fp32:
            out.append(None)
        B = d["x"].shape[0]
        absb = {k: np.abs(v) for k, v in out[0].items()}
        if B > 1:
            yall = torch.from_numpy(d["labels"]).to(device)
            N = int((yall != 255).sum())
            full = dict(masks)
            absb = None
            for b in range(B):
                for k in full:
                    masks[k] = full[k][b:b + 1]
                P = O.params_from_state(st, dtype=torch.float64, device=device)
                lg = O.forward(P, torch.from_numpy(d["x"][b:b + 1]).to(device, torch.float64), cfg)
                (F.cross_entropy(lg, yall[b:b + 1], ignore_index=255, reduction="sum") / N).backward()
                gb = {k: np.abs(v.grad.cpu().numpy()) for k, v in P.items()}
                absb = gb if absb is None else {k: absb[k] + gb[k] for k in absb}
            for k in full:
                masks[k] = full[k]
            masks.update(full)
    finally:
        O.conv_in_lrelu, O.maxpool = orig, orig_pool
    return out[0], out[1], nflip[0], absb


def _oracle_stages(P, x, cfg):
    """Intermediates of the oracle forward (channel-first), keyed like spff_saved_tensor."""
    S = {}

    def blk(name, inp):
        a, b = ("pre", "body") if cfg.novel else ("b1", "b2")
        y1 = F.conv3d(inp, P[f"{name}.{a}.0.weight"], None, padding=(1, 1, 1))
        a1 = F.leaky_relu(F.instance_norm(y1, weight=P[f"{name}.{a}.1.weight"],
                                          bias=P[f"{name}.{a}.1.bias"], eps=1e-5), 0.01)
        y2 = F.conv3d(a1, P[f"{name}.{b}.0.weight"], None, padding=(1, 1, 1))
        z = F.leaky_relu(F.instance_norm(y2, weight=P[f"{name}.{b}.1.weight"],
                                         bias=P[f"{name}.{b}.1.bias"], eps=1e-5), 0.01)
        if cfg.novel and cfg.efilm:
            z = O.energy_film(P, name + ".efilm", z)
        if cfg.novel and cfg.fgate:
            z = O.fourier_gate(P, name + ".fgate", z, cfg.learn_phase)
        S[name + ".y1"], S[name + ".a1"], S[name + ".y2"] = y1, a1, y2
        return z

    pool = lambda t: F.max_pool3d(t, (1, 2, 2))  # noqa: E731
    up = lambda t, n: F.conv_transpose3d(t, P[n + ".weight"], P[n + ".bias"], stride=(1, 2, 2))  # noqa: E731
    e1 = O._post(P, blk("enc1", x), 0, cfg); S["enc1.out"] = e1; S["pool1"] = pool(e1)
    e2 = O._post(P, blk("enc2", S["pool1"]), 1, cfg); S["enc2.out"] = e2; S["pool2"] = pool(e2)
    e3 = O._post(P, blk("enc3", S["pool2"]), 2, cfg); S["enc3.out"] = e3; S["pool3"] = pool(e3)
    b = O._post(P, blk("bott", S["pool3"]), 3, cfg); S["bott.out"] = b
    S["up3"] = up(b, "up3"); d3 = blk("dec3", torch.cat([S["up3"], e3], 1)); S["dec3.out"] = d3
    S["up2"] = up(d3, "up2"); d2 = blk("dec2", torch.cat([S["up2"], e2], 1)); S["dec2.out"] = d2
    S["up1"] = up(d2, "up1"); d1 = blk("dec1", torch.cat([S["up1"], e1], 1)); S["dec1.out"] = d1
    return S


@pytest.mark.parametrize("name", ["fx2_ns_base8", "fx3_fgate_even_b2", "fx3b_fgate_odd_b2"])
def test_stagewise_forward(name):
    """Localises a forward mismatch to the first diverging stage."""
    d = load(name)
    cfg = cfg_of(d["meta"])
    P = O.params_from_state(state_of(d), requires_grad=False)
    x = torch.from_numpy(d["x"])
    with torch.no_grad():
        S = _oracle_stages(P, x, cfg)
    core = load_core(d)
    core(x.to(DEV)).sum().backward()  # grad-mode forward -> training plan holds the stages
    plan = core._plan
    # the bottleneck / decoder outputs are applied by their GEMM consumers and not stored:
    # store them too for this view, and run the forward again
    plan.debug_set(1, 1)
    core(x.to(DEV)).sum().backward()
    order = ["enc1.y1", "enc1.a1", "enc1.y2", "enc1.out", "pool1", "enc2.out", "pool2", "enc3.out",
             "pool3", "bott.y1", "bott.out", "up3", "dec3.y1", "dec3.out", "up2", "dec2.out", "up1",
             "dec1.y1", "dec1.out"]
    report = []
    for k in order:
        r = S[k]
        mine = plan.saved(k).cpu().numpy()
        rr = r.permute(0, 2, 3, 4, 1).reshape(-1, r.shape[1]).numpy()
        e = float(np.abs(mine - rr).max()) / max(1e-6, float(np.abs(rr).max()))
        report.append((k, e))
    print("\n".join(f"  {k:10s} rel {e:.2e}" for k, e in report))
    bad = [(k, e) for k, e in report if e > 1e-4]
    assert not bad, f"first diverging stage: {bad[0]}"


@pytest.mark.parametrize("in_ch,K,base,mth", [(72, 40, 40, "f16x3"), (72, 40, 40, "f32"),
                                              (3, 100, 16, "bf16x6")])
def test_module_contract_generality(in_ch, K, base, mth):
    """VERDICT r03 missing #2: settings the registry never uses but the reference's module
    contract accepts (models.py:1558-1560) -- in_ch > 64, K > 32 (up to SPFF_MAX_CLASSES)
    and a base that is a multiple of 8 but not a power of two (channels 40/80/160/320, SE
    hidden 4/5/10/20).  Engine vs the oracle (pinned to the reference by the fixtures,
    including the reference-generated fx5_k40_base24): logits within 1e-3, argmax outside
    near-ties, loss, and every gradient against the kink-consistent fp64 oracle."""
    _engine_vs_oracle(in_ch, K, base, mth)


@pytest.mark.parametrize("in_ch,K,base,mth", [(5, 13, 32, "f16x3"), (5, 20, 32, "f32"),
                                              (5, 13, 64, "bf16x6"), (5, 32, 64, "f16x3")])
def test_streaming_head(in_ch, K, base, mth):
    """The streaming 1x1x1 head (gemm.hip k_head_fwd_s / k_head_dgrad_s: Cin = base 32 or 64,
    K <= 32; K <= 16 and 17..32 instantiations): logits, loss and every gradient (the head's
    and, through its input gradient, the network's) against the oracle as above."""
    _engine_vs_oracle(in_ch, K, base, mth)


@pytest.mark.parametrize("D,se,specse,mth", [(256, True, True, "f16x3"), (257, True, True, "f32"),
                                               (256, False, True, "f16x3"),
                                               (257, True, False, "f32")])
def test_gate_channel_split_path(D, se, specse, mth):
    """The channel-split gate kernels (gates.hip k_gfs_* / k_gbs_*, taken for C x D >= 8192):
    depth 256 / 257 at base 32 puts every level on them (level 0: 32 x 256 = 8192), with
    even and odd D (the FourierGate's Nyquist bin), and with the channel SE or the spectral
    SE off (the kernels' sw0 / specse branches).  Engine vs the oracle as below."""
    _engine_vs_oracle(5, 13, 32, mth, shape=(2, D, 8, 8), se=se, specse=specse)


def _engine_vs_oracle(in_ch, K, base, mth, shape=(1, 4, 16, 16), se=True, specse=True):
    from innovative3D.synthetic import synthetic_batch
    from innovative3D.weightgen import synth_state
    B, D, H, W = shape
    core = M.build_spct_energyfilm_fourier(num_classes=K, base=base, in_channels=in_ch,
                                           use_se=se, use_specse=specse)
    for b in core._blocks():
        b.fgate._ensure_mask(D, "cpu")
    st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=31,
                     mask_jitter=0.25)
    core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    core = core.to(DEV)
    core.math = mth
    x, y = synthetic_batch(B, in_ch, D, H, W, num_classes=K, ignore_frac=0.03, seed=32)
    logits = core(x.to(DEV))
    loss, conf = Hh.ce_dice_with_confusion(logits, y.to(DEV), K, 255)
    loss.backward()
    torch.cuda.synchronize()
    cfg = O.SpffCfg(in_ch=in_ch, num_classes=K, base=base, se=se, specse=specse)
    P = O.params_from_state({k: v for k, v in st.items() if not k.endswith("._mask")},
                            requires_grad=False)
    with torch.no_grad():
        ref = O.forward(P, x, cfg)
        ref_loss = float(O.ce_plus_macro_dice(ref, y, K)[0])
    lg = logits.detach().cpu().numpy()
    err = float(np.abs(lg - ref.numpy()).max())
    flips = lg.argmax(1) != ref.numpy().argmax(1)
    print(f"in_ch {in_ch} K {K} base {base} {mth}: max|dlogit| {err:.2e}, flips {int(flips.sum())}, "
          f"loss {float(loss):.7f} vs {ref_loss:.7f}")
    assert err <= 1e-3
    assert not (flips & ~near_tie_mask(ref.numpy(), 2 * err)).any()
    assert math.isclose(float(loss), ref_loss, rel_tol=1e-5)
    assert int(conf[:, K].sum()) == 0
    masks = engine_branch_masks(core, tuple(x.shape), st, cfg)
    ref64, ref32, nflip, absb = oracle_grads_st(cfg, st, x.numpy(), y.numpy(), masks)
    named = dict(core.named_parameters(remove_duplicate=False))
    check_grads({k: named[k].grad for k in ref64}, ref64, ref32, absb, st, mth)


@pytest.mark.parametrize("case", ["fx3b_fgate_odd_b2", "registry_2x5x8x64x64"])
def test_oracle_device_evaluation_matches_cpu(case):
    """The full-size gradient checks (tests/test_gpu_baseline_sizes.py, the world-8
    sharded test) evaluate the fp64 oracle through PyTorch's own fp64 device kernels
    instead of the CPU: pin that evaluation to the CPU one -- the same restatement, the
    same inputs, fp64 on both sides -- on a reference fixture (FourierGate at odd D,
    batch 2) and on a registry-layout (K 13, base 32) batch at 64^2 with the engine's
    own branch decisions forced on both (tests/_kink.forced_branches)."""
    from _kink import forced_branches
    if case.startswith("fx"):
        d = load(case)
        cfg, st = cfg_of(d["meta"]), state_of(d)
        x, y = torch.from_numpy(d["x"]), torch.from_numpy(d["labels"])
        masks = None
    else:
        from innovative3D.synthetic import synthetic_batch
        from innovative3D.weightgen import synth_state
        core = M.build_spct_energyfilm_fourier(num_classes=13, base=32, in_channels=5)
        for b in core._blocks():
            b.fgate._ensure_mask(8, "cpu")
        st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=3)
        cfg = O.SpffCfg(in_ch=5, num_classes=13, base=32)
        x, y = synthetic_batch(2, 5, 8, 64, 64, 13, ignore_frac=0.01, seed=3)
        core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
        core = core.to(DEV)
        lg = core(x.to(DEV))
        Hh.ce_dice_with_confusion(lg, y.to(DEV), 13, 255)[0].backward()
        torch.cuda.synchronize()
        masks = engine_branch_masks(core, tuple(x.shape), st, cfg)
        del core, lg
    st = {k: v for k, v in st.items() if not k.endswith("._mask")}
    out = []
    for dev in ("cpu", DEV):
        P = O.params_from_state(st, dtype=torch.float64, device=dev)
        if masks is None:
            lg, loss, _ce, _dice = O.fwd_bwd(P, x.to(dev, torch.float64), y.to(dev), cfg)
        else:
            with forced_branches(masks):
                lg, loss, _ce, _dice = O.fwd_bwd(P, x.to(dev, torch.float64), y.to(dev), cfg)
        out.append((lg.cpu(), float(loss), {k: v.grad.cpu() for k, v in P.items()}))
    (lc, lsc, gc), (ld, lsd, gd) = out
    e = float((lc - ld).abs().max()) / float(lc.abs().max())
    print(f"{case}: fp64 oracle on {DEV} vs cpu: logits {e:.2e} of max, loss {lsc:.15f} vs {lsd:.15f}")
    assert e <= 1e-12 and abs(lsc - lsd) <= 1e-12 * abs(lsc)
    worst = 0.0
    for k in gc:
        r = float((gc[k] - gd[k]).norm()) / max(float(gc[k].norm()), 1e-300)
        worst = max(worst, r)
        assert r <= 1e-8, f"{k}: {r:.2e}"
    print(f"  worst gradient rel L2 {worst:.2e}")


@pytest.mark.parametrize("mth", ["f16x3", "f32"])
def test_pool_fold_bitwise(mth):
    """the encoder blocks' output gradient formed by its readers (PoolAdd:
    skip gradient + the MaxPool backward of the pooled gradient, read by the tail reduction
    and the IN-backward apply) against the k_maxpool_bwd_add pass it replaced (debug key 2
    = 0).  Same sum in the same order: every parameter gradient bitwise equal."""
    from innovative3D.synthetic import synthetic_batch
    from innovative3D.weightgen import synth_state
    K = 13
    core = M.build_spct_energyfilm_fourier(num_classes=K, base=16, in_channels=5)
    for b in core._blocks():
        b.fgate._ensure_mask(8, "cpu")
    st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=5)
    core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    core = core.to(DEV)
    core.math = mth
    x, y = synthetic_batch(2, 5, 8, 32, 48, num_classes=K, ignore_frac=0.02, seed=6)
    x, y = x.to(DEV), y.to(DEV)
    grads = []
    for fold in (1, 0):
        for p in core.parameters():
            p.grad = None
        logits = core(x)
        core._plan.debug_set(2, fold)
        loss, _conf = Hh.ce_dice_with_confusion(logits, y, K, 255)
        loss.backward()
        torch.cuda.synchronize()
        grads.append({k: p.grad.detach().clone() for k, p in core.named_parameters()
                      if p.grad is not None})
    core._plan.debug_set(2, 1)
    assert grads[0].keys() == grads[1].keys() and len(grads[0]) > 20
    for k in grads[0]:
        assert torch.equal(grads[0][k], grads[1][k]), k


@pytest.mark.parametrize("mth", ["f16x3", "bf16x6"])
@pytest.mark.parametrize("shape", [(2, 8, 32, 48), (1, 5, 24, 40)])
def test_fused_in_backward_sums(mth, shape):
    """conv1's InstanceNorm-backward sums (sum dr, sum dr xhat) formed in the epilogue of the
    input-gradient conv that writes da1 (conv3d_x.hip BStat) against the RED_BWD_IN
    slab_reduce pass they replace (debug key 3 = 0).  Same terms, another summation order
    (per tile then fp64 over tiles, vs per (b, c, d) slab then fp64 over d): every parameter
    gradient within 1e-4 of its tensor's max (observed <= 2.3e-5, bf16x6 on the ragged
    case); the forward is untouched (logits bitwise).
    The ragged case (D = 5, H = 24: partial tiles) checks the epilogue's row masking."""
    from innovative3D.synthetic import synthetic_batch
    from innovative3D.weightgen import synth_state
    K = 13
    B, D, H, W = shape
    core = M.build_spct_energyfilm_fourier(num_classes=K, base=16, in_channels=5)
    for b in core._blocks():
        b.fgate._ensure_mask(D, "cpu")
    st = synth_state([(k, tuple(v.shape)) for k, v in core.state_dict().items()], seed=9)
    core.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    core = core.to(DEV)
    core.math = mth
    x, y = synthetic_batch(B, 5, D, H, W, num_classes=K, ignore_frac=0.02, seed=10)
    x, y = x.to(DEV), y.to(DEV)
    grads, logits = [], []
    for fused in (1, 0):
        for p in core.parameters():
            p.grad = None
        lg = core(x)
        core._plan.debug_set(3, fused)
        loss, _conf = Hh.ce_dice_with_confusion(lg, y, K, 255)
        loss.backward()
        torch.cuda.synchronize()
        logits.append(lg.detach().clone())
        grads.append({k: p.grad.detach().clone() for k, p in core.named_parameters()
                      if p.grad is not None})
    core._plan.debug_set(3, 1)
    assert torch.equal(logits[0], logits[1])
    worst = max(float((grads[0][k] - grads[1][k]).abs().max() /
                      grads[1][k].abs().max().clamp_min(1e-30)) for k in grads[1])
    print(f"fused IN-backward sums {mth} {shape}: worst gradient difference {worst:.2e} of max|g|")
    assert worst <= 1e-4, worst
