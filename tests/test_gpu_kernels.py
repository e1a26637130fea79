"""Per-kernel numerics on the MI355X: every HIP op against a plain PyTorch fp32 CPU reference of
the same op (through the C ABI via the ops wrappers).

Tolerances: convolutions / GEMMs use 3xBF16 split arithmetic (per-product relative error ~1e-5,
fp32 accumulation), checked at <= 2e-4 norm-wise relative error; memory-bound fp32 kernels
(GroupNorm, softmax, losses, Adam) at <= 1e-5.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CONV_TOL = 2e-4
FP32_TOL = 1e-5


def rel(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def cl(t, dev):
    return t.to(dev).contiguous(memory_format=torch.channels_last)


CONV_CASES = [
    # n, cin, cout, h, w, k, stride, pads(t,l,b,r), upsample
    (2, 32, 32, 8, 8, 3, 1, (1, 1, 1, 1), False),
    (2, 64, 128, 7, 7, 3, 1, (1, 1, 1, 1), False),
    (3, 32, 32, 15, 15, 3, 2, (0, 0, 1, 1), False),   # Downsample, odd size
    (2, 64, 64, 14, 14, 3, 2, (0, 0, 1, 1), False),   # Downsample 14 -> 7
    (2, 32, 32, 7, 7, 3, 1, (1, 1, 1, 1), True),      # Upsample 7 -> 14
    (2, 3, 32, 28, 28, 3, 1, (1, 1, 1, 1), False),    # conv_in, cin = 3
    (2, 6, 16, 16, 16, 3, 1, (1, 1, 1, 1), False),    # conditional conv_in, cin = 6
    (2, 64, 3, 16, 16, 3, 1, (1, 1, 1, 1), False),    # conv_out, cout = 3
    (2, 32, 1, 12, 12, 3, 1, (1, 1, 1, 1), False),    # conv_out, cout = 1
    (4, 128, 64, 8, 8, 1, 1, (0, 0, 0, 0), False),    # nin_shortcut 1x1
    (2, 96, 48, 9, 9, 3, 1, (1, 1, 1, 1), False),     # K-permuted order with 3 chunks per tap
    (2, 48, 96, 9, 9, 3, 1, (1, 1, 1, 1), False),     # Cin % 32 != 0: reference K order
    # production-size launches: 256x256 / 256x128 tiles, XCD remap, split-K wgrad over many splits
    (64, 256, 256, 32, 32, 3, 1, (1, 1, 1, 1), False),
    (64, 256, 128, 16, 16, 3, 1, (1, 1, 1, 1), True),  # Upsample 16 -> 32
    (64, 128, 128, 64, 64, 3, 2, (0, 0, 1, 1), False),  # Downsample 64 -> 32
    # sub-pixel Upsample: scalar-gather path (cin 3), non-square, Cin % 32 != 0, mid-size 256x256 tiles
    (2, 3, 8, 5, 6, 3, 1, (1, 1, 1, 1), True),
    (2, 48, 40, 6, 9, 3, 1, (1, 1, 1, 1), True),
    (16, 512, 256, 8, 8, 3, 1, (1, 1, 1, 1), True),
    # stride-2 input gradient by parity class: symmetric pad, non-square, 4x4 (PatchGAN), 1x1 (empty classes)
    (2, 32, 64, 10, 12, 3, 2, (1, 1, 1, 1), False),
    (2, 16, 32, 16, 16, 4, 2, (1, 1, 1, 1), False),
    (2, 32, 16, 8, 8, 1, 2, (0, 0, 0, 0), False),
    (2, 6, 8, 8, 8, 3, 2, (0, 0, 1, 1), False),
    # skinny-N 128x16 tiles (>= 512 tiles): conv_out forward (cout 3), conv_in input gradient (cin 6)
    (64, 64, 3, 32, 32, 3, 1, (1, 1, 1, 1), False),
    (64, 6, 64, 32, 32, 3, 1, (1, 1, 1, 1), False),
    # direct small-channel weight gradient (cin, cout in {32, 64}): c3 level shapes, odd / non-square images,
    # more bands than workgroups (persistent loop)
    (3, 64, 32, 28, 28, 3, 1, (1, 1, 1, 1), False),
    (2, 64, 32, 14, 14, 3, 1, (1, 1, 1, 1), False),
    (2, 32, 32, 9, 11, 3, 1, (1, 1, 1, 1), False),
    (600, 32, 32, 7, 5, 3, 1, (1, 1, 1, 1), False),
    # under-filled launches that the planner splits over K (mvae_conv2d_ws_nhwc): c2's 7x7 level at 512 channels,
    # a 2048 -> 512 narrowing conv; both fwd and dgrad split
    (64, 512, 512, 7, 7, 3, 1, (1, 1, 1, 1), False),
    (8, 1024, 256, 8, 8, 3, 1, (1, 1, 1, 1), False),
]


def torch_conv(x, w, b, stride, pads, ups):
    if ups:
        x = F.interpolate(x, scale_factor=2.0, mode="nearest")
    t, l, bo, r = pads
    x = F.pad(x, (l, r, t, bo))
    return F.conv2d(x, w, b, stride=stride)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(dev, case):
    from medvae_disentangled_multimodal_amd import ops
    n, ci, co, h, w, k, s, pads, ups = case
    g = torch.Generator().manual_seed(hash(case) % 1000)
    x = torch.randn(n, ci, h, w, generator=g)
    wt = torch.randn(co, ci, k, k, generator=g) / math.sqrt(ci * k * k)
    b = torch.randn(co, generator=g) * 0.1
    xr, wr, br = x.clone().requires_grad_(), wt.clone().requires_grad_(), b.clone().requires_grad_()
    yr = torch_conv(xr, wr, br, s, pads, ups)
    res = torch.randn(yr.shape, generator=g)
    (yr + res).mul(torch.linspace(-1, 1, yr.numel()).view(yr.shape)).sum().backward()

    geom = ops.ConvGeom(k, k, s, pads[0], pads[1], pads[2], pads[3], ups)
    xd = cl(x, dev).requires_grad_()
    wd = cl(wt, dev).requires_grad_()
    bd = b.to(dev).requires_grad_()
    yd = ops.conv2d(xd, wd, bd, geom, residual=cl(res, dev))
    assert yd.shape == yr.shape
    assert rel(yd, yr + res) < CONV_TOL
    yd.mul(torch.linspace(-1, 1, yd.numel(), device=dev).view(yd.shape)).sum().backward()
    assert rel(xd.grad, xr.grad) < CONV_TOL
    assert rel(wd.grad, wr.grad) < CONV_TOL
    # bias grad = column sum of dY, referenced in float64 (the fp32 CPU conv backward itself drifts
    # by ~1e-3 relative at 65k pixels); absolute error relative to the size of dY
    db_ref = torch.linspace(-1, 1, yr.numel()).view(yr.shape).double().sum((0, 2, 3))
    scale = float(yr.numel()) ** 0.5 + float(db_ref.abs().max())
    assert float((bd.grad.cpu().double() - db_ref).abs().max()) < 1e-5 * scale
    # flat-buffer path: weight + bias gradients accumulated in place by the fused wgrad kernel
    wm = cl(wt, dev).requires_grad_()
    bm = b.to(dev).requires_grad_()
    wm._mvae_main_grad = torch.full_like(wm, 0.5, memory_format=torch.channels_last)
    bm._mvae_main_grad = torch.full_like(bm, 0.25)
    ym = ops.conv2d(cl(x, dev), wm, bm, geom, residual=cl(res, dev))
    ym.mul(torch.linspace(-1, 1, ym.numel(), device=dev).view(ym.shape)).sum().backward()
    assert wm.grad is None and bm.grad is None
    assert rel(wm._mvae_main_grad - 0.5, wr.grad) < CONV_TOL
    assert float((bm._mvae_main_grad.cpu().double() - 0.25 - db_ref).abs().max()) < 1e-5 * scale


@pytest.mark.parametrize("n,ci,co,h", [(64, 512, 512, 7), (8, 1024, 256, 8), (32, 256, 512, 7)])
def test_conv_splitk_matches_unsplit(dev, n, ci, co, h, monkeypatch):
    """The split-K form of an under-filled conv (fwd and input gradient) is taken and agrees with the unsplit launch
    and with float64 torch."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    assert _lib.query("mvae_conv2d_split_workspace_bytes", n, ci, co, 3, 3, h, h) > 0
    assert _lib.query("mvae_conv2d_split_workspace_bytes", n, co, ci, 3, 3, h, h) > 0
    g = torch.Generator().manual_seed(n + ci + co)
    x = torch.randn(n, ci, h, h, generator=g)
    wt = torch.randn(co, ci, 3, 3, generator=g) / math.sqrt(ci * 9)
    b = torch.randn(co, generator=g) * 0.1
    res = torch.randn(n, co, h, h, generator=g)
    dy = torch.randn(n, co, h, h, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)
    y64 = F.conv2d(x.double(), wt.double(), b.double(), padding=1) + res.double()
    dx64 = torch.nn.grad.conv2d_input(x.shape, wt.double(), dy.double(), padding=1)
    outs = {}
    for on in (True, False):
        monkeypatch.setattr(ops, "CONV_SPLITK", on)
        y = ops.conv2d_forward_raw(cl(x, dev), cl(wt, dev), b.to(dev), cl(res, dev), geom)
        dx = ops.conv2d_dgrad_raw(cl(dy, dev), cl(wt, dev), x.shape, geom)
        torch.cuda.synchronize()
        assert rel(y, y64) < CONV_TOL and rel(dx, dx64) < CONV_TOL
        outs[on] = (y.cpu(), dx.cpu())
    assert rel(outs[True][0], outs[False][0]) < 1e-4 and rel(outs[True][1], outs[False][1]) < 1e-4


@pytest.mark.parametrize("ci,co,h,w,beta", [(32, 32, 28, 28, 0.0), (64, 32, 14, 14, 1.0), (32, 64, 14, 14, 0.5),
                                              (64, 64, 9, 11, 0.0)])
def test_wgrad_direct_capi_channel_pairs(dev, ci, co, h, w, beta):
    """mvae_conv2d_wgrad_direct_nhwc for every (cin, cout) pair it accepts (ops routes only cout 32 to it): dw and
    dbias accumulate with beta, against a float64 reference."""
    from medvae_disentangled_multimodal_amd import _lib
    n = 3
    g = torch.Generator().manual_seed(ci * 3 + co + h)
    x = torch.randn(n, h, w, ci, generator=g)
    dy = torch.randn(n, h, w, co, generator=g)
    dw0 = torch.randn(co, 3, 3, ci, generator=g)
    db0 = torch.randn(co, generator=g)
    xr = x.double().permute(0, 3, 1, 2)
    dyr = dy.double().permute(0, 3, 1, 2)
    wr = torch.zeros(co, ci, 3, 3, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wr, padding=1).mul(dyr).sum().backward()
    exp_dw = beta * dw0.double() + wr.grad.permute(0, 2, 3, 1)
    exp_db = beta * db0.double() + dyr.sum((0, 2, 3))
    xd, dyd, dwd, dbd = x.to(dev), dy.to(dev), dw0.to(dev), db0.to(dev)
    ws = torch.empty(_lib.query("mvae_conv2d_wgrad_direct_workspace_bytes", n, h, w, ci, co), dtype=torch.uint8,
                     device=dev)
    _lib.call("mvae_conv2d_wgrad_direct_nhwc", dyd.data_ptr(), xd.data_ptr(), dwd.data_ptr(), dbd.data_ptr(),
              float(beta), n, h, w, ci, co, 0, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rel(dwd, exp_dw) < CONV_TOL
    assert rel(dbd, exp_db) < 1e-5


@pytest.mark.parametrize("case", [c for c in CONV_CASES if c[2] % 4 == 0 and not (c[5] == 1 and c[6] == 1) and not c[8]])
def test_conv_backward_with_presplit_dy(dev, case, monkeypatch):
    """The conv's output gradient handed to both backward GEMMs pre-split (ops.split_dy -> dgrad A operand with
    MVAE_CONV_XSPLIT / stride-2 classes / upsample 4x4 form, wgrad dY^T operand with MVAE_CONV_DYSPLIT and the
    fused bias sums from hi + lo): the same tolerances as the fp32-operand path, on every geometry."""
    from medvae_disentangled_multimodal_amd import ops
    monkeypatch.setattr(ops, "DY_SPLIT_MIN", 0)
    monkeypatch.setattr(ops, "DY_SPLIT", True)
    seen = []
    orig = ops._lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    monkeypatch.setattr(ops._lib, "call", spy)
    test_conv_fwd_dgrad_wgrad(dev, case)
    assert "mvae_split_bf16" in seen


@pytest.mark.parametrize("case", CONV_CASES[:14] + CONV_CASES[18:22])
def test_conv_exact_fp32_mode(dev, case):
    """Math mode 2 (the trainer's precision "32-exact"; the discriminator's default): every conv GEMM on the
    f32-input MFMA -- fwd / dgrad / wgrad agree with float64 to fp32 accumulation error (5e-6 norm-wise; the
    3xBF16 path sits at 1e-5..3e-5), and no pre-split operand is formed."""
    from medvae_disentangled_multimodal_amd import ops
    n, ci, co, h, w, k, s, pads, ups = case
    g = torch.Generator().manual_seed(5 + hash(case) % 1000)
    x = torch.randn(n, ci, h, w, generator=g)
    wt = torch.randn(co, ci, k, k, generator=g) / math.sqrt(ci * k * k)
    b = torch.randn(co, generator=g) * 0.1
    xr, wr, br = x.double().requires_grad_(), wt.double().requires_grad_(), b.double().requires_grad_()
    yr = torch_conv(xr, wr, br, s, pads, ups)
    gy = torch.randn(yr.shape, generator=g)
    yr.backward(gy.double())
    geom = ops.ConvGeom(k, k, s, pads[0], pads[1], pads[2], pads[3], ups)
    with ops.math_scope(2):
        xd = cl(x, dev).requires_grad_()
        wd = cl(wt, dev).requires_grad_()
        bd = b.to(dev).requires_grad_()
        yd = ops.conv2d(xd, wd, bd, geom)
        yd.backward(cl(gy, dev))
    assert ops._MATH[0] == 0
    assert rel(yd, yr) < 5e-6
    assert rel(xd.grad, xr.grad) < 5e-6
    assert rel(wd.grad, wr.grad) < 5e-6
    assert rel(bd.grad, br.grad) < 5e-6


def test_attention_gemm_exact_fp32_mode(dev):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(2)
    q, k_, v = (torch.randn(4, 64, 8, 8, generator=g) for _ in range(3))
    qr, kr, vr = (t.double().requires_grad_() for t in (q, k_, v))
    b, c, hh, ww = q.shape
    qq, kk, vv = (t.reshape(b, c, hh * ww).permute(0, 2, 1) for t in (qr, kr, vr))
    p = torch.softmax(qq @ kk.transpose(1, 2) * c ** -0.5, dim=2)
    o_r = (p @ vv).permute(0, 2, 1).reshape(b, c, hh, ww)
    go = torch.randn(o_r.shape, generator=g)
    o_r.backward(go.double())
    with ops.math_scope(2):
        qd, kd, vd = (cl(t, dev).requires_grad_() for t in (q, k_, v))
        o = ops.attention_core(qd, kd, vd)
        o.backward(cl(go, dev))
    assert rel(o, o_r) < 5e-6
    for a, r in ((qd, qr), (kd, kr), (vd, vr)):
        assert rel(a.grad, r.grad) < 5e-6


def test_split_bf16_layout(dev):
    """mvae_split_bf16: per 4 fp32 values hi0..hi3 lo0..lo3 (bf16), hi = RNE(x), lo = RNE(x - hi)."""
    from medvae_disentangled_multimodal_amd import _lib
    x = torch.randn(4096, generator=torch.Generator().manual_seed(3)) * 10.0
    xd = x.to(dev)
    y = torch.empty(4096 * 4, dtype=torch.uint8, device=dev)
    _lib.call("mvae_split_bf16", xd.data_ptr(), y.data_ptr(), 4096, torch.cuda.current_stream().cuda_stream)
    hl = y.view(torch.bfloat16).view(-1, 2, 4).cpu()
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    assert torch.equal(hl[:, 0].flatten(), hi) and torch.equal(hl[:, 1].flatten(), lo)
    assert float(((hi.float() + lo.float()) - x).abs().max() / x.abs().max()) < 2 ** -15


@pytest.mark.parametrize("split", [0, 1])
def test_weight_prep_split_layouts(dev, split):
    """Weight re-layouts with split output equal the fp32 re-layout split afterwards."""
    from medvae_disentangled_multimodal_amd import _lib
    g = torch.Generator().manual_seed(11)
    co, ci = 64, 32
    w = cl(torch.randn(co, ci, 3, 3, generator=g), dev)
    st = torch.cuda.current_stream().cuda_stream
    for name, n_out, args in (("mvae_conv_weight_transpose", 9 * ci * co, (co, 3, 3, ci)),
                              ("mvae_conv_weight_upsample_dgrad", 16 * ci * co, (co, ci)),
                              ("mvae_conv_weight_upsample_fwd", 16 * ci * co, (co, ci))):
        ref = torch.empty(n_out, device=dev)
        _lib.call(name, w.data_ptr(), ref.data_ptr(), *args, 0, st)
        out = torch.empty(n_out, device=dev)
        _lib.call(name, w.data_ptr(), out.data_ptr(), *args, split, st)
        if split:
            exp = torch.empty(n_out, device=dev)
            _lib.call("mvae_split_bf16", ref.data_ptr(), exp.data_ptr(), n_out, st)
            assert torch.equal(out.view(torch.int32), exp.view(torch.int32)), name
        else:
            assert torch.equal(out, ref), name


@pytest.mark.parametrize("drop,co", [(0.0, 32), (0.25, 32), (0.0, 3)])
def test_groupnorm_split_output_feeds_conv(dev, drop, co):
    """GroupNorm(+SiLU, dropout) written pre-split for a following conv (MVAE_CONV_XSPLIT): the bytes are
    the split of the fp32 output, and the conv (fwd + weight grad) matches the conv of the fp32 output
    (co = 3: Decoder.conv_out, whose weight gradient runs on the small-cout kernel)."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    g = torch.Generator().manual_seed(21)
    n, c, h = 2, 64, 12
    x = cl(torch.randn(n, c, h, h, generator=g) * 2 + 0.5, dev)
    gam = (torch.rand(c, generator=g) + 0.5).to(dev)
    bet = (torch.randn(c, generator=g) * 0.1).to(dev)
    y32 = ops.group_norm(x, gam, bet, 32, 1e-6, True, drop, 77)
    ys = ops.group_norm(x, gam, bet, 32, 1e-6, True, drop, 77, for_conv=True)
    assert getattr(ys, ops.XSPLIT_ATTR, False)
    exp = torch.empty_like(y32)
    _lib.call("mvae_split_bf16", y32.data_ptr(), exp.data_ptr(), y32.numel(), torch.cuda.current_stream().cuda_stream)
    assert torch.equal(ys.view(torch.int32), exp.view(torch.int32))
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1)
    w = cl(torch.randn(co, c, 3, 3, generator=g) / 24.0, dev)
    wa, wb = w.clone().requires_grad_(), w.clone().requires_grad_()
    ya = ops.conv2d(y32, wa, None, geom)
    yb = ops.conv2d(ys, wb, None, geom)
    assert rel(yb, ya) < 1e-5
    gy = torch.randn(ya.shape, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    ya.backward(gy)
    yb.backward(gy)
    assert rel(wb.grad, wa.grad) < 1e-5


def test_upsample_gather_mode_matches_subpixel(dev):
    """The direct gather form of Upsample's conv (mvae_conv2d_nhwc mode 1: 9 taps on the upsampled grid)
    and the sub-pixel form (4 parity classes of 2x2 convs) give the same result."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    g = torch.Generator().manual_seed(5)
    n, ci, co, h, w = 3, 64, 32, 7, 9
    x = cl(torch.randn(n, ci, h, w, generator=g), dev)
    wt = cl(torch.randn(co, ci, 3, 3, generator=g) / 24.0, dev)
    b = torch.randn(co, generator=g).to(dev)
    ref = torch_conv(x.cpu(), wt.cpu(), b.cpu(), 1, (1, 1, 1, 1), True)
    y1 = torch.empty((n, co, 2 * h, 2 * w), device=dev).contiguous(memory_format=torch.channels_last)
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("mvae_conv2d_nhwc", x.data_ptr(), wt.data_ptr(), b.data_ptr(), None, y1.data_ptr(), n, h, w, ci, co,
              3, 3, 1, 1, 1, 2 * h, 2 * w, 1, st)
    y2 = ops.conv2d_forward_raw(x, wt, b, None, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, True))
    assert rel(y1, ref) < CONV_TOL and rel(y2, ref) < CONV_TOL
    assert rel(y1, y2) < CONV_TOL


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("m,n,k,batch", [(64, 64, 32, 3), (49, 100, 37, 2), (256, 128, 512, 1), (3, 200, 4096, 1)])
def test_gemm_strided_batched(dev, ta, tb, m, n, k, batch):
    from medvae_disentangled_multimodal_amd import _lib
    g = torch.Generator().manual_seed(m * 7 + n + k)
    A = torch.randn(batch, k, m, generator=g) if ta else torch.randn(batch, m, k, generator=g)
    B = torch.randn(batch, n, k, generator=g) if tb else torch.randn(batch, k, n, generator=g)
    C0 = torch.randn(batch, m, n, generator=g)
    bias = torch.randn(n, generator=g)
    res = torch.randn(batch, m, n, generator=g)
    opA = A.transpose(1, 2) if ta else A
    opB = B.transpose(1, 2) if tb else B
    ref = 0.5 * (opA @ opB) + bias + res + 0.25 * C0
    Ad, Bd, Cd = A.to(dev), B.to(dev), C0.to(dev).clone()
    bd, rd = bias.to(dev), res.to(dev)
    ws = torch.empty(_lib.query("mvae_gemm_workspace_bytes", m, n, k, batch) + 16, dtype=torch.uint8, device=dev)
    lda = m if ta else k
    ldb = k if tb else n
    _lib.call("mvae_gemm_strided_batched", ta, tb, m, n, k, 0.5, Ad.data_ptr(), lda, m * k, Bd.data_ptr(), ldb,
              n * k, 0.25, Cd.data_ptr(), n, m * n, batch, bd.data_ptr(), rd.data_ptr(), n, m * n,
              ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream)
    assert rel(Cd, ref) < CONV_TOL


@pytest.mark.parametrize("n,c,h,w,silu,drop", [(2, 32, 8, 8, False, 0.0), (2, 64, 7, 7, True, 0.0),
                                                (3, 128, 16, 16, True, 0.0), (2, 2048, 4, 4, True, 0.0),
                                                (2, 16, 5, 5, False, 0.0)])
def test_group_norm_silu(dev, n, c, h, w, silu, drop):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(c + h)
    x = torch.randn(n, c, h, w, generator=g) * 2 + 0.5
    gamma = 1 + 0.2 * torch.randn(c, generator=g)
    beta = 0.1 * torch.randn(c, generator=g)
    G = min(32, c)
    xr, gr, br = x.clone().requires_grad_(), gamma.clone().requires_grad_(), beta.clone().requires_grad_()
    yr = F.group_norm(xr, G, gr, br, eps=1e-6)
    if silu:
        yr = yr * torch.sigmoid(yr)
    wgt = torch.randn(yr.shape, generator=g)
    (yr * wgt).sum().backward()
    xd, gd, bd = cl(x, dev).requires_grad_(), gamma.to(dev).requires_grad_(), beta.to(dev).requires_grad_()
    yd = ops.group_norm(xd, gd, bd, G, 1e-6, silu)
    assert rel(yd, yr) < FP32_TOL
    (yd * cl(wgt, dev)).sum().backward()
    assert rel(xd.grad, xr.grad) < 1e-4
    assert rel(gd.grad, gr.grad) < 1e-4
    assert rel(bd.grad, br.grad) < 1e-4


def _gn_raw(path, x, gamma, beta, dy, add, groups, silu, drop, seed, y_split=0):
    """One fwd + bwd through the C ABI on the selected GroupNorm path (0 auto/resident, 1 streaming)."""
    from medvae_disentangled_multimodal_amd import _lib
    n, h, w, c = x.shape
    st = torch.cuda.current_stream().cuda_stream
    _lib.call("mvae_set_group_norm_path", path)
    try:
        ws = torch.empty(_lib.query("mvae_group_norm_workspace_bytes", n, h * w, c), dtype=torch.uint8,
                         device=x.device)
        y = torch.empty_like(x)
        mean = torch.empty(n * groups, device=x.device)
        rstd = torch.empty_like(mean)
        _lib.call("mvae_group_norm_fwd_nhwc", x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), y.data_ptr(),
                  mean.data_ptr(), rstd.data_ptr(), n, h * w, c, groups, 1e-6, int(silu), float(drop), seed, y_split,
                  ws.data_ptr(), ws.numel(), st)
        dx = torch.empty_like(x)
        dg = torch.full((c,), 0.5, device=x.device)  # accumulated into (+=)
        db = torch.full((c,), -0.25, device=x.device)
        _lib.call("mvae_group_norm_bwd_nhwc", x.data_ptr(), dy.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                  mean.data_ptr(), rstd.data_ptr(), dx.data_ptr(), add.data_ptr() if add is not None else None,
                  dg.data_ptr(), db.data_ptr(), n, h * w, c, groups, int(silu), float(drop), seed, ws.data_ptr(),
                  ws.numel(), st)
        torch.cuda.synchronize()
    finally:
        _lib.call("mvae_set_group_norm_path", 0)
    return y, mean, rstd, dx, dg, db


# the c3 (28/14/7 at hidden 32) and c2 (hidden 128) levels, whose h*w is not a multiple of 32 (no conv-epilogue
# statistics): auto selects the register-resident one-pass kernels (backward of larger tensors: the two-pass
# unit kernel); checked against float64 torch and against the streaming kernels (dropout masks identical: same
# counter hash)
@pytest.mark.parametrize("n,c,h,silu,drop,add", [(3, 32, 28, True, 0.0, True), (3, 64, 14, True, 0.1, False),
                                                  (2, 128, 7, False, 0.0, True), (2, 256, 14, True, 0.0, False),
                                                  (2, 512, 7, True, 0.1, True), (2, 128, 28, True, 0.0, False),
                                                  (2, 2048, 4, True, 0.0, True), (5, 96, 9, True, 0.0, False),
                                                  # two-pass unit backward (64x64 / 48x48: too many rows to hold)
                                                  (2, 256, 64, True, 0.1, True), (2, 512, 48, True, 0.0, False)])
def test_group_norm_resident_matches_streaming_and_float64(dev, n, c, h, silu, drop, add):
    g = torch.Generator().manual_seed(c * 7 + h)
    G = min(32, c)
    x = (torch.randn(n, h, h, c, generator=g) * 1.5 + 0.3).to(dev)
    gamma = (1 + 0.2 * torch.randn(c, generator=g)).to(dev)
    beta = (0.1 * torch.randn(c, generator=g)).to(dev)
    dy = torch.randn(n, h, h, c, generator=g).to(dev)
    ad = torch.randn(n, h, h, c, generator=g).to(dev) if add else None
    res = _gn_raw(0, x, gamma, beta, dy, ad, G, silu, drop, 77)
    stream = _gn_raw(1, x, gamma, beta, dy, ad, G, silu, drop, 77)
    for a, b in zip(res, stream):
        assert rel(a, b) < 1e-5
    assert torch.equal(res[0] == 0, stream[0] == 0)  # same dropout mask
    if drop == 0.0:
        xr = x.double().permute(0, 3, 1, 2).cpu().requires_grad_()
        gr, br = gamma.double().cpu().requires_grad_(), beta.double().cpu().requires_grad_()
        yr = F.group_norm(xr, G, gr, br, eps=1e-6)
        if silu:
            yr = yr * torch.sigmoid(yr)
        (yr * dy.double().permute(0, 3, 1, 2).cpu()).sum().backward()
        y, _, _, dx, dg, db = res
        assert rel(y.permute(0, 3, 1, 2).cpu(), yr) < FP32_TOL
        exp_dx = xr.grad + (ad.double().permute(0, 3, 1, 2).cpu() if add else 0.0)
        assert rel(dx.permute(0, 3, 1, 2).cpu(), exp_dx) < 1e-5
        assert rel(dg.cpu() - 0.5, gr.grad) < 1e-5
        assert rel(db.cpu() + 0.25, br.grad) < 1e-5
    # bitwise reproducible run to run
    again = _gn_raw(0, x, gamma, beta, dy, ad, G, silu, drop, 77)
    for a, b in zip(res, again):
        assert torch.equal(a, b)


def test_dropout_mask_statistics_and_grad_consistency(dev):
    from medvae_disentangled_multimodal_amd import ops
    x = cl(torch.randn(4, 64, 16, 16), dev).requires_grad_()
    gamma = torch.ones(64, device=dev, requires_grad=True)
    beta = torch.zeros(64, device=dev, requires_grad=True)
    y = ops.group_norm(x, gamma, beta, 32, 1e-6, True, 0.1, 1234)
    y0 = ops.group_norm(x.detach(), gamma.detach(), beta.detach(), 32, 1e-6, True, 0.0, 0)
    dropped = (y == 0) & (y0 != 0)
    frac = dropped.float().mean().item()
    assert 0.08 < frac < 0.12
    kept = ~dropped
    assert torch.allclose(y[kept], y0[kept] / 0.9, rtol=1e-5, atol=1e-6)
    # gradient uses the same (recomputed) mask: zero grad flows through dropped units only
    y.sum().backward()
    x2 = x.detach().clone().requires_grad_()
    y2 = ops.group_norm(x2, gamma.detach(), beta.detach(), 32, 1e-6, True, 0.0, 0)
    (y2 * kept.float() / 0.9).sum().backward()
    assert rel(x.grad, x2.grad) < 1e-5


def test_attention_core(dev):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(5)
    b, c, h, w = 2, 64, 7, 7
    q, k, v = [torch.randn(b, c, h, w, generator=g) for _ in range(3)]
    qr, kr, vr = [t.clone().requires_grad_() for t in (q, k, v)]
    n = h * w
    s = torch.bmm(qr.reshape(b, c, n).permute(0, 2, 1), kr.reshape(b, c, n)) * c ** -0.5
    a = torch.softmax(s, 2)
    o = torch.bmm(vr.reshape(b, c, n), a.permute(0, 2, 1)).reshape(b, c, h, w)
    wgt = torch.randn(o.shape, generator=g)
    (o * wgt).sum().backward()
    qd, kd, vd = [cl(t, dev).requires_grad_() for t in (q, k, v)]
    od = ops.attention_core(qd, kd, vd)
    assert rel(od, o) < CONV_TOL
    (od * cl(wgt, dev)).sum().backward()
    for dd, rr in ((qd, qr), (kd, kr), (vd, vr)):
        assert rel(dd.grad, rr.grad) < 5e-4


def test_reparam_kl_mse(dev):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(9)
    h = torch.randn(3, 16, 7, 7, generator=g)
    eps = torch.randn(3, 8, 7, 7, generator=g)
    hr = h.clone().requires_grad_()
    mr, lr_ = torch.chunk(hr, 2, 1)
    zr = mr + eps * torch.exp(0.5 * lr_)
    s = torch.exp(0.5 * lr_)
    kl = (0.5 * (s * s + mr * mr - 1 - torch.log(s * s))).mean()
    x = torch.randn(3, 8, 7, 7, generator=g)
    mse = F.mse_loss(zr, x)
    (kl * 0.7 + mse * 1.3).backward()
    hd = cl(h, dev).requires_grad_()
    md, ld = torch.chunk(hd, 2, 1)
    zd = ops.reparameterize(md, ld, cl(eps, dev))
    kd = ops.kl_standard_normal_mean(md, ld)
    sd = ops.mse_mean(zd, cl(x, dev))
    assert rel(zd, zr) < FP32_TOL
    assert abs(kd.item() - kl.item()) < 1e-6 * abs(kl.item()) + 1e-7
    assert abs(sd.item() - mse.item()) < 1e-6 * abs(mse.item()) + 1e-7
    (kd * 0.7 + sd * 1.3).backward()
    assert rel(hd.grad, hr.grad) < FP32_TOL


def test_multi_tensor_adam_matches_torch(dev):
    from medvae_disentangled_multimodal_amd.optim import FlatParameters, FusedAdam
    torch.manual_seed(0)
    shapes = [(8, 4, 3, 3), (8,), (70000,), (5, 5)]
    for decoupled, wd, betas in ((True, 1e-2, (0.9, 0.999)), (False, 1e-3, (0.5, 0.999))):
        mod = torch.nn.Module()
        ps = [torch.nn.Parameter(torch.randn(s)) for s in shapes]
        for i, p in enumerate(ps):
            mod.register_parameter(f"p{i}", p)
        ref = [p.detach().clone().requires_grad_() for p in ps]
        opt_ref = (torch.optim.AdamW if decoupled else torch.optim.Adam)(ref, lr=1e-2, betas=betas, weight_decay=wd)
        flat = FlatParameters(mod, dev)
        opt = FusedAdam(flat, lr=1e-2, betas=betas, weight_decay=wd, decoupled=decoupled, max_grad_norm=1.0)
        for it in range(3):
            grads = [torch.randn(s) * (3.0 if it == 0 else 0.3) for s in shapes]
            if it == 1:
                grads[3][0, 0] = float("nan")  # non-finite -> whole tensor's grad zeroed
            for r, gr in zip(ref, grads):
                r.grad = gr.clone()
            for r in ref:
                if not torch.isfinite(r.grad).all():
                    r.grad.zero_()
            torch.nn.utils.clip_grad_norm_(ref, 1.0)
            opt_ref.step()
            flat.zero_grad()
            for p, gr in zip(flat.params, grads):
                p._mvae_main_grad.copy_(gr.to(dev))
            opt.step()
        for p, r in zip(flat.params, ref):
            assert rel(p, r) < 1e-6


@pytest.mark.parametrize("cin,cout,attn", [(64, 64, False), (64, 128, False), (64, 64, True)])
def test_block_input_gradient_branches_summed_in_groupnorm(dev, cin, cout, attn):
    """ResnetBlock (identity residual and nin_shortcut) and AttnBlock: the residual-side gradient of the
    block input is parked in a GradSink and summed inside norm1's GroupNorm backward; the input gradient
    must equal the float64 torch functional reference (encoder_decoder.py:68-170)."""
    from medvae_disentangled_multimodal_amd import encoder_decoder as E
    torch.manual_seed(3)
    blk = (E.AttnBlock(cin) if attn else E.ResnetBlock(in_channels=cin, out_channels=cout)).to(dev)
    x = torch.randn(2, cin, 8, 8)
    xd = cl(x, dev).requires_grad_(True)
    y = blk(xd)
    gy = torch.randn(y.shape)
    y.backward(cl(gy, dev))
    P = {k: v.detach().double().cpu() for k, v in blk.state_dict().items()}
    xr = x.double().requires_grad_(True)
    if attn:
        h = F.group_norm(xr, 32, P["norm.weight"], P["norm.bias"], eps=1e-6)
        q, k, v = (F.conv2d(h, P[f"{n}.weight"], P[f"{n}.bias"]) for n in "qkv")
        b, c, hh, ww = q.shape
        w_ = torch.softmax(torch.bmm(q.reshape(b, c, -1).permute(0, 2, 1), k.reshape(b, c, -1)) * c ** -0.5, dim=2)
        o = torch.bmm(v.reshape(b, c, -1), w_.permute(0, 2, 1)).reshape(b, c, hh, ww)
        yr = xr + F.conv2d(o, P["proj_out.weight"], P["proj_out.bias"])
    else:
        h = F.silu(F.group_norm(xr, 32, P["norm1.weight"], P["norm1.bias"], eps=1e-6))
        h = F.conv2d(h, P["conv1.weight"], P["conv1.bias"], padding=1)
        h = F.silu(F.group_norm(h, 32, P["norm2.weight"], P["norm2.bias"], eps=1e-6))
        h = F.conv2d(h, P["conv2.weight"], P["conv2.bias"], padding=1)
        sc = xr if cin == cout else F.conv2d(xr, P["nin_shortcut.weight"], P["nin_shortcut.bias"])
        yr = sc + h
    yr.backward(gy.double())
    assert rel(y, yr) < CONV_TOL
    assert rel(xd.grad, xr.grad) < 1e-3


@pytest.mark.parametrize("n,c,co,h,res", [(4, 64, 128, 16, False), (8, 128, 256, 8, True), (16, 256, 256, 32, True)])
def test_conv_epilogue_groupnorm_statistics(dev, n, c, co, h, res, monkeypatch):
    """conv2d(gn_stats=True) emits {sum, sum sq} per 32 pixels x 4 channels from the GEMM epilogue and the
    following GroupNorm(+SiLU) finalizes from them (no statistics pass): same output as the two-pass
    GroupNorm of the same conv output; an in-place change of the conv output drops the statistics.
    (The statistics launch is never split over K; the plain launch is held unsplit too, for bitwise equality.)"""
    from medvae_disentangled_multimodal_amd import ops
    monkeypatch.setattr(ops, "CONV_SPLITK", False)
    g = torch.Generator().manual_seed(7)
    x = cl(torch.randn(n, c, h, h, generator=g), dev)
    w = cl(torch.randn(co, c, 3, 3, generator=g) / math.sqrt(9 * c), dev)
    b = (torch.randn(co, generator=g) * 0.3 + 0.5).to(dev)
    r = cl(torch.randn(n, co, h, h, generator=g), dev) if res else None
    gam = (torch.rand(co, generator=g) + 0.5).to(dev)
    bet = (torch.randn(co, generator=g) * 0.1).to(dev)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1)
    y0 = ops.conv2d(x, w, b, geom, residual=r)
    y1 = ops.conv2d(x, w, b, geom, residual=r, gn_stats=True)
    assert getattr(y1, ops.GN_PART_ATTR, None) is not None
    assert torch.equal(y0, y1)
    ref = ops.group_norm(y0, gam, bet, 32, 1e-6, True)
    out = ops.group_norm(y1, gam, bet, 32, 1e-6, True)
    assert not hasattr(y1, ops.GN_PART_ATTR)
    assert rel(out, ref) < 1e-5
    # against float64 torch as well
    t = F.silu(F.group_norm(y0.double().cpu(), 32, gam.double().cpu(), bet.double().cpu(), eps=1e-6))
    assert rel(out, t) < 1e-5
    y2 = ops.conv2d(x, w, b, geom, residual=r, gn_stats=True)
    y2.mul_(2.0)  # stale statistics must not be used
    assert rel(ops.group_norm(y2, gam, bet, 32, 1e-6, True),
               F.silu(F.group_norm(y2.double().cpu(), 32, gam.double().cpu(), bet.double().cpu(), eps=1e-6))) < 1e-5


@pytest.mark.parametrize("n,c,co,h,silu", [
    (4, 64, 128, 16, True),     # 2 channels per group: not eligible, the two-pass backward must run
    (8, 256, 64, 8, True), (2, 128, 32, 32, False), (16, 256, 256, 32, True),
    (2, 256, 256, 64, True),    # c4 level 0 (64x64, C=256)
    (2, 512, 512, 32, True),    # c4 level 1
    (2, 1024, 1024, 16, True),  # c4 level 2
    (2, 2048, 2048, 8, True),   # c4 level 3 / mid
    (4, 128, 128, 28, True),    # c2 level 0 (28x28: 784 % 32 == 16, not eligible)
])
@pytest.mark.parametrize("wino", [False, True], ids=["gemm", "winograd"])
def test_groupnorm_backward_partials_from_conv_dgrad(dev, n, c, co, h, silu, wino, monkeypatch):
    """GroupNorm(+SiLU) -> conv: the conv's input-gradient GEMM emits the GroupNorm backward partials
    (mvae_conv2d_dgrad_gnbwd_nhwc) and the GroupNorm backward skips its reduction pass
    (mvae_group_norm_bwd_part_nhwc) -- exactly when the shape is eligible (H*W % 32 == 0 and C/G % 4 == 0).
    dx / dgamma / dbeta / dW equal the unfused path (1e-5) and float64 torch autograd (1e-4; 2e-4 when the conv runs in
    Winograd F(4x4, 3x3) form, whose output transform emits the partials instead of the GEMM epilogue)."""
    from medvae_disentangled_multimodal_amd import ops
    monkeypatch.setattr(ops, "WINOGRAD", wino)
    monkeypatch.setattr(ops, "WINOGRAD_MIN_MACS", 0.0)
    wino_used = wino and ops._wino_ok(ops.ConvGeom(3, 3, 1, 1, 1, 1, 1), n, h, h, co, c)
    if wino and not wino_used:
        pytest.skip("not a Winograd geometry")
    producer = "mvae_winograd_output_gnbwd" if wino_used else "mvae_conv2d_dgrad_gnbwd_nhwc"
    eligible = (h * h) % 32 == 0 and (c // 32) % 4 == 0
    g = torch.Generator().manual_seed(11 + c)
    x0 = torch.randn(n, c, h, h, generator=g) * 1.5 + 0.3
    gam0 = torch.rand(c, generator=g) + 0.5
    bet0 = torch.randn(c, generator=g) * 0.1
    w0 = torch.randn(co, c, 3, 3, generator=g) / math.sqrt(9 * c)
    gy = torch.randn(n, co, h, h, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1)

    def run(fused):
        prev = ops.GN_BWD_FUSED
        ops.GN_BWD_FUSED = fused
        try:
            x = cl(x0, dev).requires_grad_()
            gam, bet = gam0.to(dev).requires_grad_(), bet0.to(dev).requires_grad_()
            w = cl(w0, dev).requires_grad_()
            y = ops.group_norm(x, gam, bet, 32, 1e-6, silu, for_conv=True)
            link = getattr(y, ops.GN_BWD_ATTR, None)
            assert (link is not None) == fused
            out = ops.conv2d(y, w, None, geom)
            seen = []
            if fused:
                orig = ops._lib.call

                def spy(name, *args):
                    seen.append(name)
                    return orig(name, *args)
                ops._lib.call = spy
            try:
                out.backward(cl(gy, dev))
            finally:
                if fused:
                    ops._lib.call = orig
            if fused and eligible:
                assert producer in seen and "mvae_group_norm_bwd_part_nhwc" in seen
                assert "mvae_group_norm_bwd_nhwc" not in seen
            elif fused:
                assert producer not in seen and "mvae_group_norm_bwd_part_nhwc" not in seen
                assert "mvae_group_norm_bwd_nhwc" in seen
            return x.grad, gam.grad, bet.grad, w.grad
        finally:
            ops.GN_BWD_FUSED = prev

    fz, un = run(True), run(False)
    for a, b in zip(fz, un):
        assert rel(a, b) < 1e-5
    xr = x0.double().requires_grad_()
    gr, br, wr = gam0.double().requires_grad_(), bet0.double().requires_grad_(), w0.double().requires_grad_()
    yr = F.group_norm(xr, 32, gr, br, eps=1e-6)
    if silu:
        yr = F.silu(yr)
    F.conv2d(yr, wr, None, 1, 1).backward(gy.double())
    for a, b in zip(fz, (xr.grad, gr.grad, br.grad, wr.grad)):
        assert rel(a, b) < (2e-4 if wino_used else 1e-4)


@pytest.mark.parametrize("n,ci,co,h,w", [(4, 64, 128, 16, 16), (2, 256, 64, 8, 32), (3, 64, 64, 64, 8), (16, 128, 256, 8, 8)])
@pytest.mark.parametrize("x_split", [False, True])
def test_wgrad_pow2_gather(dev, n, ci, co, h, w, x_split):
    """The shift-and-mask im2col gather of the weight gradient (B_WGRAD_P2: stride-1 'same' 3x3 convs at power-of-two
    H, W -- every c4 / c5 level), plain and on a pre-split 3xBF16 input (the GroupNorm -> conv edge), non-square images
    included: dW and the fused bias gradient against float64."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    g = torch.Generator().manual_seed(n * ci + h * w)
    x = torch.randn(n, ci, h, w, generator=g)
    dy = torch.randn(n, co, h, w, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)
    xd, dyd = cl(x, dev), cl(dy, dev)
    if x_split:
        xs = torch.empty_like(xd)
        _lib.call("mvae_split_bf16", xd.data_ptr(), xs.data_ptr(), xd.numel(), ops._stream(xd))
        xd = xs
    dw = torch.zeros(co, ci, 3, 3, device=dev).contiguous(memory_format=torch.channels_last)
    db = torch.zeros(co, device=dev)
    ops.conv2d_wgrad_raw(dyd, xd, dw, 0.0, geom, db=db, x_split=x_split)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(x.double(), (co, ci, 3, 3), dy.double(), padding=1)
    assert rel(dw, ref) < CONV_TOL
    assert rel(db, dy.double().sum((0, 2, 3))) < 1e-5
