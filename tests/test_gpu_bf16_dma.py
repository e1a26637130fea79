"""Convolutions on DMA-staged operands: bf16-mixed on packed bf16 operands (MVAE_CONV_BF16: LDS-DMA main loop of the
implicit GEMM, 64-deep K-tiles, source-swizzled ROW images) and the fp32-class 3xBF16 mode on planar hi / lo bf16
operands (MVAE_CONV_PLANAR, 32-deep K-tiles; the size rule ops.PLANAR_MIN_MACS is lowered to 0 here so the small
edge cases take that path). The edge cases of that loader: channel counts that are multiples of 8 but not
of 64 (K-tiles straddle filter taps, no K permutation), ragged pixel tails (M not a multiple of any tile), the
stride-2 Downsample forward and its input gradient by parity class, the sub-pixel Upsample forward and its 4x4
stride-2 input gradient, and a 1x1-tap conv. Reference: float64 on the bf16-rounded GEMM operands (forward: x, w;
input gradient: dy, w), so only fp32 accumulation differs -- tolerance 2e-5 (tests/test_gpu_c5.py). The same
launches through the register-staged bf16 loop (ops.BF16_DMA off) agree to the same tolerance. 3xBF16: float64 on the
fp32 operands at the fp32-class conv tolerance 2e-4 (tests/test_gpu_kernels.py CONV_TOL), and the planar path against
the register-staged 3xBF16 loop (same K order, same split) at 2e-6."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
TOL = 2e-5


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def bf(t):
    return t.bfloat16().double()


def rel(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


# n, cin, cout, h, w, k, stride, pads (t, l, b, r), upsample
CASES = [
    (2, 40, 24, 12, 10, 3, 1, (1, 1, 1, 1), False),    # cin % 64 != 0: K-tiles straddle taps
    (3, 128, 72, 9, 7, 3, 1, (1, 1, 1, 1), False),     # ragged M (189 pixels), N = 72
    (2, 64, 128, 16, 16, 3, 2, (0, 0, 1, 1), False),   # Downsample: pad (0, 1), stride 2
    (2, 256, 256, 16, 16, 3, 1, (1, 1, 1, 1), False),  # K permutation on (cin % 64 == 0)
    (2, 64, 96, 8, 8, 3, 1, (1, 1, 1, 1), True),       # Upsample 8 -> 16 (sub-pixel forward, 4x4 input gradient)
    (2, 48, 32, 6, 6, 2, 1, (0, 0, 1, 1), False),      # 2x2 kernel, asymmetric pad
]


def _run(dev, case, dma, prec="bf16-mixed"):
    from medvae_disentangled_multimodal_amd import ops
    n, ci, co, h, w, k, s, pads, ups = case
    g = torch.Generator().manual_seed(ci * 13 + co + h)
    x = torch.randn(n, ci, h, w, generator=g)
    wt = torch.randn(co, ci, k, k, generator=g) / math.sqrt(ci * k * k)
    b = torch.randn(co, generator=g) * 0.1
    geom = ops.ConvGeom(k, k, s, *pads, ups)
    xd = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    wd = wt.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    bd = b.to(dev).requires_grad_()
    saved = (ops.BF16_DMA, ops.PLANAR_DMA, ops.PLANAR_MIN_MACS)
    ops.BF16_DMA = ops.PLANAR_DMA = dma
    ops.PLANAR_MIN_MACS = 0
    prev = ops.set_precision(prec)
    try:
        y = ops.conv2d(xd, wd, bd, geom)
        dy = torch.randn(y.shape, generator=g)
        y.backward(dy.to(dev).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(prev)
        ops.BF16_DMA, ops.PLANAR_DMA, ops.PLANAR_MIN_MACS = saved
    return x, wt, b, dy, y.detach(), xd.grad, geom, wd.grad, bd.grad


def _subpixel_kernels(w):
    """class kernels of nearest-x2 + 3x3 (pad 1) as fp32 tap sums, rounded to bf16 (the GEMM operands)."""
    groups = {0: ((0,), (1, 2)), 1: ((0, 1), (2,))}
    ks = {}
    for ph in (0, 1):
        for pw in (0, 1):
            k = torch.zeros(w.shape[0], w.shape[1], 2, 2)
            for a, rs in enumerate(groups[ph]):
                for c, ss in enumerate(groups[pw]):
                    k[:, :, a, c] = sum(w[:, :, r, s] for r in rs for s in ss)
            ks[(ph, pw)] = k.bfloat16().double()
    return ks


@pytest.mark.parametrize("case", CASES)
def test_bf16_dma_conv_fwd_dgrad(dev, case):
    x, wt, b, dy, y, dx, geom, _, _ = _run(dev, case, True)
    n, ci, co, h, w, k, s, pads, ups = case
    xr = bf(x).requires_grad_()
    if ups:
        ks = _subpixel_kernels(wt)
        yr = xr.new_zeros(n, co, 2 * h, 2 * w)
        for (ph, pw), kk in ks.items():
            yr[:, :, ph::2, pw::2] = F.conv2d(F.pad(xr, (1 - pw, pw, 1 - ph, ph)), kk)
        yr = yr + b.double().view(1, -1, 1, 1)
    else:
        pt, pl, pb, pr = pads
        yr = F.conv2d(F.pad(xr, (pl, pr, pt, pb)), bf(wt), b.double(), stride=s)
    assert rel(y, yr) < TOL
    # (Upsample: the input gradient runs as a stride-2 4x4 conv whose tap-summed weights are the same fp32 partial sums
    # as the class kernels, rounded to bf16)
    yr.backward(bf(dy))
    assert rel(dx, xr.grad) < TOL


@pytest.mark.parametrize("case", CASES[:4])
def test_bf16_dma_matches_register_staged_loop(dev, case):
    _, _, _, _, y1, dx1, _, _, _ = _run(dev, case, True)
    _, _, _, _, y0, dx0, _, _, _ = _run(dev, case, False)
    assert rel(y1, y0) < TOL
    assert rel(dx1, dx0) < TOL


@pytest.mark.parametrize("case", CASES)
def test_planar_3xbf16_conv_fwd_dgrad_wgrad(dev, case):
    x, wt, b, dy, y, dx, geom, dw, db = _run(dev, case, True, "32")
    n, ci, co, h, w, k, s, pads, ups = case
    xr = x.double().requires_grad_()
    wr = wt.double().requires_grad_()
    xin = F.interpolate(xr, scale_factor=2.0, mode="nearest") if ups else xr
    pt, pl, pb, pr = pads
    yr = F.conv2d(F.pad(xin, (pl, pr, pt, pb)), wr, b.double(), stride=s)
    yr.backward(dy.double())
    assert rel(y, yr) < 2e-4
    assert rel(dx, xr.grad) < 2e-4
    assert rel(dw, wr.grad) < 2e-4
    assert rel(db, dy.double().sum((0, 2, 3))) < 1e-5
    # the register-staged 3xBF16 loop: same operand split, same K order
    _, _, _, _, y0, dx0, _, dw0, _ = _run(dev, case, False, "32")
    assert rel(y, y0) < 2e-6
    assert rel(dx, dx0) < 2e-6
    assert rel(dw, dw0) < 2e-6
