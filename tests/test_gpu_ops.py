"""Per-op parity of the HIP kernels vs the CPU oracle (torch-CPU fp32 ops that
the reference itself calls).  Marked gpu: run on the MI355X box."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from innovative3D import _engine as E
import innovative3D.helpers as Hh
from oracle import spff_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cl(t):  # [B,C,D,H,W] -> [B,D,H,W,C]
    return t.permute(0, 2, 3, 4, 1).contiguous()


def _ncdhw(t):  # [B,D,H,W,C] -> [B,C,D,H,W]
    return t.permute(0, 4, 1, 2, 3).contiguous()


CONV_CASES = [
    # B, D, H, W, cin, cout, ksd
    (2, 5, 16, 32, 8, 32, 3),
    (1, 3, 8, 16, 5, 32, 3),     # first layer, Cin=5 padded to ld 8
    (1, 4, 16, 16, 32, 64, 3),
    (1, 2, 8, 8, 64, 128, 3),
    (1, 3, 8, 16, 16, 8, 3),     # base-8 nets: Cout < 32
    (2, 4, 8, 16, 32, 32, 1),    # ksd = 1
    (1, 5, 24, 40, 16, 16, 3),   # ragged tiles (H, W not multiples of the tile)
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv3d_fwd_dgrad_wgrad(case):
    B, D, H, W, cin, cout, ksd = case
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, cin, D, H, W, generator=g)
    w = torch.randn(cout, cin, ksd, 3, 3, generator=g) / math.sqrt(cin * ksd * 9)
    dy = torch.randn(B, cout, D, H, W, generator=g)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    y = F.conv3d(xr, wr, None, padding=(ksd // 2, 1, 1))
    y.backward(dy)
    ldx = (cin + 7) // 8 * 8
    xcl = torch.zeros(B, D, H, W, ldx)
    xcl[..., :cin] = _cl(x)
    xcl = xcl.to(DEV)
    wd = w.to(DEV)
    ws = torch.empty(E.lib().spff_conv3d_ws_bytes(B, D, H, W, cin, cout, ksd), dtype=torch.uint8,
                     device=DEV)
    L, p, st = E.lib(), E._ptr, E._stream(torch.device(DEV))
    yg = torch.empty(B, D, H, W, cout, device=DEV)
    E.check(L.spff_conv3d_fwd(p(xcl), ldx, p(wd), p(yg), B, D, H, W, cin, cout, ksd, p(ws), st), "fwd")
    dyg = _cl(dy).to(DEV)
    dwg = torch.empty_like(wd)
    E.check(L.spff_conv3d_wgrad(p(xcl), ldx, p(dyg), p(dwg), B, D, H, W, cin, cout, ksd, p(ws), st),
            "wgrad")
    torch.cuda.synchronize()
    ref = _cl(y.detach())
    assert float((yg.cpu() - ref).abs().max()) <= 2e-5 * float(ref.abs().max()) + 1e-6
    assert float((dwg.cpu() - wr.grad).abs().max()) <= 2e-5 * float(wr.grad.abs().max()) + 1e-6
    if cin % 4 == 0:
        dxg = torch.empty(B, D, H, W, cin, device=DEV)
        E.check(L.spff_conv3d_dgrad(p(dyg), p(wd), p(dxg), B, D, H, W, cin, cout, ksd, p(ws), st), "dgrad")
        torch.cuda.synchronize()
        refx = _cl(xr.grad)
        assert float((dxg.cpu() - refx).abs().max()) <= 2e-5 * float(refx.abs().max()) + 1e-6


SPLIT_CASES = [
    # B, D, H, W, cin, cout, ksd  (H, W >= 16: the split-bf16 kernel's tile)
    (2, 5, 16, 32, 8, 32, 3),
    (1, 3, 16, 16, 5, 32, 3),     # first layer, Cin=5 padded to ld 8
    (1, 4, 16, 16, 32, 64, 3),
    (1, 3, 32, 48, 64, 128, 3),
    (1, 3, 16, 16, 16, 8, 3),     # Cout < 32
    (2, 4, 16, 16, 32, 32, 1),    # ksd = 1
    (1, 5, 24, 40, 16, 16, 3),    # ragged tiles
]


@pytest.mark.parametrize("math_mode", ["bf16x6", "bf16x3", "f16x3"])
@pytest.mark.parametrize("case", SPLIT_CASES)
def test_conv3d_split_bf16(case, math_mode, amp=(1.0, 1.0, 1.0)):
    """fwd / dgrad / wgrad on the bf16 matrix cores with the exact 3-plane (2-plane)
    operand split, against an fp64 conv.  bf16x6 and f16x3 (scaled fp16 planes) must be
    as accurate as the fp32 MFMA path (error within 4x of it); bf16x3 within 3e-5 of
    max|ref|.  amp: magnitudes of x, w, dy (f16x3's operand scaling)."""
    B, D, H, W, cin, cout, ksd = case
    mth = E.MATH_NAMES[math_mode]
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, cin, D, H, W, generator=g) * amp[0]
    w = torch.randn(cout, cin, ksd, 3, 3, generator=g) / math.sqrt(cin * ksd * 9) * amp[1]
    dy = torch.randn(B, cout, D, H, W, generator=g) * amp[2]
    y64 = F.conv3d(x.double(), w.double(), None, padding=(ksd // 2, 1, 1))
    dx64 = torch.nn.grad.conv3d_input(x.shape, w.double(), dy.double(), padding=(ksd // 2, 1, 1))
    dw64 = torch.nn.grad.conv3d_weight(x.double(), w.shape, dy.double(), padding=(ksd // 2, 1, 1))
    ldx = (cin + 7) // 8 * 8
    xcl = torch.zeros(B, D, H, W, ldx)
    xcl[..., :cin] = _cl(x)
    xcl, wd, dyg = xcl.to(DEV), w.to(DEV), _cl(dy).to(DEV)
    L, p, st = E.lib(), E._ptr, E._stream(torch.device(DEV))
    ws = torch.empty(L.spff_conv3d_ws_bytes(B, D, H, W, cin, cout, ksd), dtype=torch.uint8,
                     device=DEV)
    out = {}
    for m in (E.MATH_F32, mth):
        yg = torch.empty(B, D, H, W, cout, device=DEV)
        E.check(L.spff_conv3d_fwd_ex(p(xcl), ldx, p(wd), p(yg), B, D, H, W, cin, cout, ksd, m,
                                     p(ws), st), "fwd")
        dxg = None
        if cin % 4 == 0:
            dxg = torch.empty(B, D, H, W, cin, device=DEV)
            E.check(L.spff_conv3d_dgrad_ex(p(dyg), p(wd), p(dxg), B, D, H, W, cin, cout, ksd, m,
                                           p(ws), st), "dgrad")
        dwg = torch.empty_like(wd)
        E.check(L.spff_conv3d_wgrad_ex(p(xcl), ldx, p(dyg), p(dwg), B, D, H, W, cin, cout, ksd, m,
                                       p(ws), st), "wgrad")
        torch.cuda.synchronize()
        out[m] = (yg.cpu().double(), None if dxg is None else dxg.cpu().double(),
                  dwg.cpu().double())
    pairs = [(0, _cl(y64)), (2, dw64)] + ([(1, _cl(dx64))] if cin % 4 == 0 else [])
    for k, ref in pairs:
        e32 = float((out[E.MATH_F32][k] - ref).abs().max())
        ex = float((out[mth][k] - ref).abs().max())
        scale = float(ref.abs().max())
        print(f"{math_mode} {case} amp={amp} op {k}: max err {ex / scale:.2e} of max|ref| "
              f"(f32 path {e32 / scale:.2e})")
        if math_mode in ("bf16x6", "f16x3"):
            assert ex <= 4 * e32 + 1e-7 * scale, (k, ex, e32)
        else:
            assert ex <= 3e-5 * scale, (k, ex, scale)


@pytest.mark.parametrize("amp", [(1e-12, 1e6, 1e-9), (3e4, 1e-5, 2e5), (1e-30, 1e-3, 1e20)])
def test_conv3d_f16x3_operand_scaling(amp):
    """f16x3 scales each operand by a power of two from its on-device max |element|: far
    outside fp16's range (1e-30 .. 1e20) it is as accurate as the fp32 MFMA path."""
    test_conv3d_split_bf16((1, 4, 16, 16, 32, 32, 3), "f16x3", amp)


@pytest.mark.parametrize("K,shape", [(13, (2, 5, 16, 16)), (9, (1, 16, 32, 32)), (2, (1, 3, 8, 8)),
                                     (100, (1, 4, 32, 33)), (128, (1, 3, 16, 16)),
                                     (13, (2, 33, 65, 67)), (4, (1, 65, 65, 66)),
                                     (3, (2, 3, 11, 13))])
def test_loss_matches_oracle(K, shape):
    """K > 64 takes the HBM confusion path (wave-aggregated atomics): labels and argmax
    skewed onto a few cells there, as segmentation labels are.  The last three: more 64-voxel
    runs than the grid has waves, so runs come from the register prefetch (loss.hip
    SPFF_LOSS_PF), with a ragged last run of 6 rows (K 13: plain copy), of 2 rows (K 4: the
    prefetch path's partial quad run) and a small ragged case."""
    g = torch.Generator().manual_seed(K)
    logits = torch.randn(shape[0], K, *shape[1:], generator=g) * 2
    y = torch.randint(0, K, shape, generator=g)
    if K > 64:
        bg = torch.rand(shape, generator=g) < 0.8
        y[bg] = 0
        logits[:, 0][bg] += 6.0
    y[torch.rand(shape, generator=g) < 0.05] = 255
    if K > 3:
        y[y == 2] = 3  # an absent class
    lr = logits.clone().requires_grad_(True)
    loss_ref, ce_ref, dice_ref = O.ce_plus_macro_dice(lr, y, K)
    loss_ref.backward()
    lg = logits.to(DEV).requires_grad_(True)
    loss, conf = Hh.ce_dice_with_confusion(lg, y.to(DEV), K, 255)
    loss.backward()
    torch.cuda.synchronize()
    assert math.isclose(float(loss), float(loss_ref), rel_tol=2e-6)
    np.testing.assert_array_equal(conf.cpu().numpy()[:, :K], O.confusion(logits, y, K, 255))
    assert float((lg.grad.cpu() - lr.grad).abs().max()) <= 1e-7
    # standalone helpers
    assert math.isclose(Hh.macro_dice_loss(lg, y.to(DEV), K), dice_ref, abs_tol=1e-12)
    met = Hh.per_class_metrics_3d(lg.detach(), y.to(DEV), K, ignore_index=255)
    ref = O.per_class_metrics_3d(logits, y, K, ignore_index=255)
    np.testing.assert_allclose(np.array(met[0]), np.array(ref[0]), rtol=1e-12, equal_nan=True)
    np.testing.assert_allclose(np.array(met[3:]), np.array(ref[3:]), rtol=1e-12, equal_nan=True)


def test_loss_all_ignored_is_nan_with_zero_grad():
    K = 4
    lg = torch.randn(1, K, 2, 4, 4, device=DEV, requires_grad=True)
    y = torch.full((1, 2, 4, 4), 255, dtype=torch.long, device=DEV)
    loss = Hh.ce_plus_macro_dice_loss(lg, y, K)
    loss.backward()
    assert math.isnan(float(loss))
    assert float(lg.grad.abs().max()) == 0.0


def _near(mask, rd, rh, rw):
    """voxels within (rd, rh, rw) of a set voxel of mask [B, D, H, W] (box dilation)"""
    m = mask.double().unsqueeze(1)
    k = torch.ones(1, 1, 2 * rd + 1, 2 * rh + 1, 2 * rw + 1, dtype=torch.float64)
    return F.conv3d(m, k, padding=(rd, rh, rw))[:, 0] > 0


@pytest.mark.parametrize("cin,cout", [(32, 32), (64, 64), (16, 16)])
def test_conv3d_f16x3_intra_tensor_range(cin, cout):
    """a few outliers 1e10 .. 1e12 x the rest inside ONE operand.
    The outputs whose receptive field excludes the outliers are judged per output
    against an fp64 conv, relative to the output's own absolute sum A_i = (|x| * |w|)_i
    (the scale of fp32 summation error), and compared with the f32 MFMA path on the same
    outputs.  Inside a tile whose halo holds an outlier, f16x3's per-(tile, chunk) scale
     flushes elements below 2^-39 of the outlier, so "away" = more than one
    tile (4 x 8 x 16 voxels) plus the halo from every outlier.  fwd: outliers in x; dgrad:
    outliers in dy; wgrad (its outputs sum over every voxel, outliers included): outliers in
    x, judged per weight against sum_v |x(v + t)| |dy(v)|."""
    B, D, H, W, ksd = 1, 12, 32, 48, 3
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, cin, D, H, W, generator=g)
    w = torch.randn(cout, cin, ksd, 3, 3, generator=g) / math.sqrt(cin * ksd * 9)
    dy = torch.randn(B, cout, D, H, W, generator=g)
    out_mask = torch.zeros(B, D, H, W, dtype=torch.bool)
    for (d, h, ww), a in zip(((2, 5, 7), (9, 26, 40), (6, 17, 3)), (1e10, 1e11, 1e12)):
        x[0, :, d, h, ww] *= a
        dy[0, :, d, h, ww] *= a
        out_mask[0, d, h, ww] = True
    far = ~_near(out_mask, 5, 9, 17)
    assert int(far.sum()) > 0.3 * far.numel()
    pad = (ksd // 2, 1, 1)
    y64 = F.conv3d(x.double(), w.double(), None, padding=pad)
    ya = F.conv3d(x.double().abs(), w.double().abs(), None, padding=pad)
    dx64 = torch.nn.grad.conv3d_input(x.shape, w.double(), dy.double(), padding=pad)
    dxa = torch.nn.grad.conv3d_input(x.shape, w.double().abs(), dy.double().abs(), padding=pad)
    # wgrad: outliers only in x (dy without them), per weight vs its absolute sum
    dy_w = torch.randn(B, cout, D, H, W, generator=g)
    dw64 = torch.nn.grad.conv3d_weight(x.double(), w.shape, dy_w.double(), padding=pad)
    dwa = torch.nn.grad.conv3d_weight(x.double().abs(), w.shape, dy_w.double().abs(), padding=pad)
    ldx = cin
    L, p, st = E.lib(), E._ptr, E._stream(torch.device(DEV))
    xcl, wd, dyg, dywg = _cl(x).to(DEV), w.to(DEV), _cl(dy).to(DEV), _cl(dy_w).to(DEV)
    ws = torch.empty(L.spff_conv3d_ws_bytes(B, D, H, W, cin, cout, ksd), dtype=torch.uint8,
                     device=DEV)
    res = {}
    for m in (E.MATH_F32, E.MATH_NAMES["f16x3"]):
        yg = torch.empty(B, D, H, W, cout, device=DEV)
        dxg = torch.empty(B, D, H, W, cin, device=DEV)
        dwg = torch.empty_like(wd)
        E.check(L.spff_conv3d_fwd_ex(p(xcl), ldx, p(wd), p(yg), B, D, H, W, cin, cout, ksd, m,
                                     p(ws), st), "fwd")
        E.check(L.spff_conv3d_dgrad_ex(p(dyg), p(wd), p(dxg), B, D, H, W, cin, cout, ksd, m,
                                       p(ws), st), "dgrad")
        E.check(L.spff_conv3d_wgrad_ex(p(xcl), ldx, p(dywg), p(dwg), B, D, H, W, cin, cout, ksd,
                                       m, p(ws), st), "wgrad")
        torch.cuda.synchronize()
        e_y = ((yg.cpu().double() - _cl(y64)).abs() / _cl(ya).clamp_min(1e-300))[far]
        e_x = ((dxg.cpu().double() - _cl(dx64)).abs() / _cl(dxa).clamp_min(1e-300))[far]
        e_w = (dwg.cpu().double() - dw64).abs() / dwa.clamp_min(1e-300)
        res[m] = (float(e_y.max()), float(e_x.max()), float(e_w.max()))
    f32, f16 = res[E.MATH_F32], res[E.MATH_NAMES["f16x3"]]
    for k, name in enumerate(("fwd", "dgrad", "wgrad")):
        print(f"cin {cin} cout {cout} {name}: max per-output error / abs-sum away from the "
              f"outliers: f16x3 {f16[k]:.2e}, f32 MFMA {f32[k]:.2e}")
    for k in range(3):
        assert f16[k] <= max(4 * f32[k], 2e-7), (k, f16, f32)


def _upconv_ref(x, w, b):
    """ConvTranspose3d(k = s = (1,2,2)) + bias in fp64 on the host: x [B,D,H,W,Cin]
    channel-last, w [Cin][Cout][1][2][2] -> y [B,D,2H,2W,Cout]"""
    xt = x.permute(0, 4, 1, 2, 3).double()
    y = torch.nn.functional.conv_transpose3d(xt, w.double(), b.double(), stride=(1, 2, 2))
    return y.permute(0, 2, 3, 4, 1).contiguous()


@pytest.mark.parametrize("cin,cout,outliers", [(64, 32, False), (128, 64, False), (32, 16, True),
                                               (64, 32, True)])
def test_upconv_gemm_arithmetics(cin, cout, outliers):
    """The up-convolution GEMMs (gemm.hip k_gemm_x forward / input gradient, k_atb_x weight
    gradient) in each arithmetic against fp64: f16x3 takes per-(tile, chunk) power-of-two
    scales of both operands (gemm_chunk_scale), bf16x6 the exact 3-plane split.  Errors per
    output relative to its absolute sum (sum |x||w|), the conv tests' measure
    (test_conv3d_f16x3_intra_tensor_range) and the same outlier regime: a few elements
    1e10 .. 1e11 above the rest in ONE operand -- x for the forward and the weight gradient,
    dy for the input gradient; the forward / input-gradient outputs that share a GEMM tile
    with an outlier row are excluded (a tile's scale flushes elements below 2^-39 of its
    largest), the weight gradient (each output a sum over every voxel, the outliers
    included) is judged on every weight."""
    L = E.lib()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(cin + cout)
    B, D, H, W = 2, 3, 24, 40
    x = torch.randn(B, D, H, W, cin, generator=g)
    w = torch.randn(cin, cout, 1, 2, 2, generator=g) * 0.1
    b = torch.randn(cout, generator=g)
    dy = torch.randn(B, D, 2 * H, 2 * W, cout, generator=g)
    dyo = dy.clone()  # the input gradient's operand (outliers here when outliers)
    far_x = torch.ones(B, D, H, W, dtype=torch.bool)
    if outliers:
        for (bb, d, h, ww), a in zip(((0, 1, 3, 5), (1, 2, 20, 33)), (1e10, 1e11)):
            x[bb, d, h, ww] *= a
            dyo[bb, d, 2 * h, 2 * ww] *= a
            far_x[bb, d, max(h - 8, 0):h + 9, :] = False  # rows sharing a GEMM tile
    y64 = _upconv_ref(x, w, b)
    ya = _upconv_ref(x.abs(), w.abs(), b.abs())
    # dgrad: dx[v][ci] = sum_{ij, co} dy[high(v, ij)][co] W[ci][co][ij]
    dyt = dyo.permute(0, 4, 1, 2, 3).double()
    dx64 = torch.nn.functional.conv3d(dyt, w.double(), stride=(1, 2, 2)).permute(0, 2, 3, 4, 1)
    dxa = torch.nn.functional.conv3d(dyt.abs(), w.double().abs(), stride=(1, 2, 2)).permute(0, 2, 3, 4, 1)
    # wgrad: dW[ci][co][ij] = sum_v x[v][ci] dy[high(v, ij)][co]
    xt = x.permute(0, 4, 1, 2, 3).double()
    dyw = dy.permute(0, 4, 1, 2, 3).double()
    ww = w.double().clone().requires_grad_(True)
    torch.nn.functional.conv_transpose3d(xt, ww, stride=(1, 2, 2)).backward(dyw)
    dw64 = ww.grad
    ww2 = w.double().clone().requires_grad_(True)
    torch.nn.functional.conv_transpose3d(xt.abs(), ww2, stride=(1, 2, 2)).backward(dyw.abs())
    dwa = ww2.grad
    db64 = dyw.sum((0, 2, 3, 4))
    ws = torch.empty(int(L.spff_upconv_ws_bytes(B, D, H, W, cin, cout)), dtype=torch.uint8,
                     device=DEV)
    p = lambda t: t.data_ptr()  # noqa: E731
    xd, wd, bd, dyd, dyod = x.to(DEV), w.to(DEV), b.to(DEV), dy.to(DEV), dyo.to(DEV)
    res = {}
    far_y = far_x.repeat_interleave(2, 2).repeat_interleave(2, 3)
    for m in (E.MATH_F32, E.MATH_BF16X6, E.MATH_F16X3):
        yg = torch.empty(B, D, 2 * H, 2 * W, cout, device=DEV)
        dxg = torch.empty(B, D, H, W, cin, device=DEV)
        dwg = torch.empty_like(wd)
        dbg = torch.empty_like(bd)
        E.check(L.spff_upconv_fwd(p(xd), p(wd), p(bd), p(yg), B, D, H, W, cin, cout, m, p(ws), st),
                "fwd")
        E.check(L.spff_upconv_dgrad(p(dyod), p(wd), p(dxg), B, D, H, W, cin, cout, m, p(ws), st),
                "dgrad")
        E.check(L.spff_upconv_wgrad(p(xd), p(dyd), p(dwg), p(dbg), B, D, H, W, cin, cout, m, p(ws),
                                    st), "wgrad")
        torch.cuda.synchronize()
        e_y = ((yg.cpu().double() - y64).abs() / ya.clamp_min(1e-300))[far_y]
        e_x = ((dxg.cpu().double() - dx64).abs() / dxa.clamp_min(1e-300))[far_x]
        e_w = (dwg.cpu().double() - dw64).abs() / dwa.clamp_min(1e-300)
        e_b = float((dbg.cpu().double() - db64).abs().max() / db64.abs().max())
        res[m] = (float(e_y.max()), float(e_x.max()), float(e_w.max()), e_b)
        print(f"upconv {cin}->{cout} outliers={outliers} math {m}: fwd {res[m][0]:.2e} dgrad "
              f"{res[m][1]:.2e} wgrad {res[m][2]:.2e} bias {res[m][3]:.2e}")
    f32 = res[E.MATH_F32]
    for m in (E.MATH_BF16X6, E.MATH_F16X3):
        for i, what in enumerate(("fwd", "dgrad", "wgrad")):
            # fp32-class: within 4x the fp32 MFMA path's error (and 1e-6 of the abs-sum)
            assert res[m][i] <= max(4 * f32[i], 1e-6), (m, what, res[m][i], f32[i])
        assert res[m][3] <= 1e-6  # the bias gradient is an fp32 column sum in every mode
