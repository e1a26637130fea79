"""Direct 3x3 stencil kernel for 32 -> 32 channel convolutions (csrc/conv_direct.hip: the c3 model's 28x28 level,
ResnetBlock convs of encoder_decoder.py:123-146): forward (bias, residual, pre-split input / weights) and input
gradient against float64 torch and against the implicit-GEMM path in the same arithmetic."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = {"32": 3e-5, "32-exact": 3e-6}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def _run(dev, x, w, b, res, go, prec, direct, presplit_x=False):
    from medvae_disentangled_multimodal_amd import ops
    prev, saved = ops.set_precision(prec), ops.DIRECT32
    ops.DIRECT32 = direct
    try:
        xd = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
        wd = w.to(dev).requires_grad_()
        bd = b.to(dev).requires_grad_()
        rd = res.to(dev).contiguous(memory_format=torch.channels_last) if res is not None else None
        g = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1)
        inp = xd
        if presplit_x:  # the GroupNorm-written pre-split operand (identity affine: y = GN(x) is what the conv sees)
            inp = ops.group_norm(xd, torch.ones(32, device=dev), torch.zeros(32, device=dev), 8, for_conv=True)
        y = ops.conv2d(inp, wd, bd, g, residual=rd)
        y.backward(go.to(dev).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
        return y, xd.grad, wd.grad, bd.grad
    finally:
        ops.restore_math_mode(prev)
        ops.DIRECT32 = saved


@pytest.mark.parametrize("prec", sorted(TOL))
@pytest.mark.parametrize("shape,resid", [((4, 32, 28, 28), True), ((3, 32, 7, 11), False), ((2, 32, 31, 5), True),
                                         ((1, 32, 60, 60), False)], ids=lambda v: str(v))
def test_direct32_matches_float64_and_gemm(dev, shape, resid, prec):
    n, c, h, w_ = shape
    g = torch.Generator().manual_seed(h * 100 + w_)
    x = torch.randn(shape, generator=g)
    w = torch.randn(32, 32, 3, 3, generator=g) / 17.0
    b = torch.randn(32, generator=g)
    res = torch.randn(n, 32, h, w_, generator=g) if resid else None
    go = torch.randn(n, 32, h, w_, generator=g)
    xr, wr, br = (t.double().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, padding=1) + (res.double() if resid else 0)
    yr.backward(go.double())
    got = _run(dev, x, w, b, res, go, prec, True)
    gemm = _run(dev, x, w, b, res, go, prec, False)
    tol = TOL[prec]
    for name, a, r, q in zip(("y", "dx", "dw", "db"), got, (yr, xr.grad, wr.grad, br.grad), gemm):
        assert _rel(a, r) < tol, (name, _rel(a, r))
        assert _rel(a, q) < tol, (name, "vs gemm", _rel(a, q))


def test_direct32_presplit_input(dev):
    """the conv input written pre-split by the GroupNorm (MVAE_CONV_XSPLIT): same result as the GEMM path"""
    shape = (3, 32, 28, 28)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(shape, generator=g)
    w = torch.randn(32, 32, 3, 3, generator=g) / 17.0
    b = torch.randn(32, generator=g)
    go = torch.randn(shape, generator=g)
    got = _run(dev, x, w, b, None, go, "32", True, presplit_x=True)
    gemm = _run(dev, x, w, b, None, go, "32", False, presplit_x=True)
    for a, q in zip(got, gemm):
        assert _rel(a, q) < 2e-5


def test_direct32_is_used(dev):
    """the c3 28x28 geometry goes through the direct kernel in both directions"""
    from medvae_disentangled_multimodal_amd import _lib
    calls = []
    real = _lib.call

    def counting(name, *args):
        calls.append(name)
        return real(name, *args)
    _lib.call = counting
    try:
        g = torch.Generator().manual_seed(1)
        _run(dev, torch.randn(2, 32, 28, 28, generator=g), torch.randn(32, 32, 3, 3, generator=g),
             torch.randn(32, generator=g), None, torch.randn(2, 32, 28, 28, generator=g), "32", True)
    finally:
        _lib.call = real
    assert calls.count("mvae_conv2d_direct32_nhwc") == 2
