"""Winograd F(2x2, 3x3) and F(4x4, 3x3) convolution (csrc/winograd.hip) against float64 references: forward with bias, residual and the
fused GroupNorm statistics, input gradient with and without the GroupNorm backward partials, pre-split (3xBF16) inputs,
both supported widths (8, 16) and non-square heights; and through ops.conv2d's dispatcher against the implicit-GEMM
path of the same layer.

Tolerance: 3xBF16 GEMM arithmetic on fp32 transforms, <= 2e-4 norm-wise relative error (the conv bar of
test_gpu_kernels.py; measured ~1e-5 for F2, ~5e-5 for F4 -- the north_star output bar is 1e-3); the fp64 statistics to
1e-5 relative."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CONV_TOL = 2e-4

# n, cin, cout, h, w
CASES = [
    (2, 64, 64, 8, 8),
    (3, 128, 64, 16, 16),
    (2, 32, 96, 12, 8),    # non-square, cin != cout
    (1, 256, 128, 4, 16),  # one tile row pair per image
    (4, 512, 512, 8, 8),   # c4-like channel count, 256-wide GEMM tiles
    (2, 64, 32, 8, 32),    # W = 32: per-segment output groups
    (1, 32, 64, 12, 64),   # W = 64: two 32-pixel segments per row
    (3, 64, 64, 7, 7),     # c2's 7x7 level: edge tiles cut (no fused statistics)
    (2, 32, 48, 14, 10),   # ragged both ways
    (1, 1024, 1024, 4, 4), # cin x cout >= 2^20: the two-pass input-gradient filter transform (m = 4)
]


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


def _split(t):
    from medvae_disentangled_multimodal_amd import _lib, ops
    s = torch.empty_like(t)
    _lib.call("mvae_split_bf16", t.data_ptr(), s.data_ptr(), t.numel(), ops._stream(t))
    return s


def _stats64(y, groups_of=4):
    """{sum, sum of squares} per 32-pixel block and 4-channel group of an NHWC float64 tensor."""
    n, c, h, w = y.shape
    t = y.permute(0, 2, 3, 1).reshape(n * h * w // 32, 32, c // groups_of, groups_of)
    return torch.stack([t.sum((1, 3)), (t * t).sum((1, 3))], -1).flatten()


@pytest.fixture(autouse=True, params=[2, 4], ids=["F2", "F4"])
def _wino_on(monkeypatch, request):
    """Every test for both output tiles: F(2x2, 3x3) and F(4x4, 3x3)."""
    from medvae_disentangled_multimodal_amd import ops
    monkeypatch.setattr(ops, "WINOGRAD", True)
    monkeypatch.setattr(ops, "WINOGRAD_MIN_C", 1)
    monkeypatch.setattr(ops, "WINOGRAD_MIN_C_WIDE", 1)
    monkeypatch.setattr(ops, "WINOGRAD_TILE", request.param)
    monkeypatch.setattr(ops, "WINOGRAD_MAX_W", 64)
    monkeypatch.setattr(ops, "WINOGRAD_MIN_MACS", 0.0)
    return request.param


@pytest.mark.parametrize("n,ci,co,h,w", CASES)
@pytest.mark.parametrize("x_split", [False, True])
def test_winograd_forward(dev, n, ci, co, h, w, x_split, monkeypatch):
    from medvae_disentangled_multimodal_amd import _lib, ops
    g = torch.Generator().manual_seed(n * ci + co + h * w)
    x = torch.randn(n, ci, h, w, generator=g)
    wt = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
    b = torch.randn(co, generator=g)
    r = torch.randn(n, co, h, w, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)
    assert ops._wino_ok(geom, n, h, w, ci, co)
    xd = cl(x, dev)
    if x_split:
        xd = _split(xd)
    blocks = ops._wino_blocks(h, w)
    part = torch.empty(n * h * w // 32 * (co // 4) * 2, device=dev, dtype=torch.float64) if blocks else None
    seen = []
    orig = _lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    monkeypatch.setattr(_lib, "call", spy)
    y = ops.conv2d_forward_raw(xd, cl(wt, dev), b.to(dev), cl(r, dev), geom, x_split=x_split, gn_part=part)
    monkeypatch.setattr(_lib, "call", orig)
    torch.cuda.synchronize()
    assert "mvae_winograd_output_transform" in seen
    ref = torch.nn.functional.conv2d(x.double(), wt.double(), b.double(), padding=1) + r.double()
    assert rel(y, ref) < CONV_TOL
    if blocks:
        assert rel(part, _stats64(y.double().cpu())) < 1e-9  # the statistics are of the stored y
        assert rel(part, _stats64(ref)) < CONV_TOL


@pytest.mark.parametrize("n,ci,co,h,w", CASES)
@pytest.mark.parametrize("dy_split", [False, True])
def test_winograd_input_gradient(dev, n, ci, co, h, w, dy_split):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(7 * n + ci + co + h)
    dy = torch.randn(n, co, h, w, generator=g)
    wt = torch.randn(co, ci, 3, 3, generator=g) / (3 * co ** 0.5)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)
    dyd = cl(dy, dev)
    dys = _split(dyd) if dy_split else None
    dx = ops.conv2d_dgrad_raw(dyd, cl(wt, dev), (n, ci, h, w), geom, dys=dys)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_input((n, ci, h, w), wt.double(), dy.double(), padding=1)
    assert rel(dx, ref) < CONV_TOL


@pytest.mark.parametrize("n,ci,co,h,w", CASES)
@pytest.mark.parametrize("split", [False, True])
def test_winograd_weight_gradient(dev, n, ci, co, h, w, split):
    """F(3x3, 2x2) weight gradient accumulating into dW (beta = 1) on plain and pre-split x / dy."""
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(3 * n + ci + 2 * co + w)
    x = torch.randn(n, ci, h, w, generator=g)
    dy = torch.randn(n, co, h, w, generator=g)
    dw0 = torch.randn(co, ci, 3, 3, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)
    xd, dyd = cl(x, dev), cl(dy, dev)
    dw = cl(dw0, dev)
    assert ops._wino_wgrad_ok(geom, xd, dyd, dw, None)
    fused = ops.conv2d_wgrad_raw(dyd, _split(xd) if split else xd, dw, 1.0, geom, x_split=split,
                                 dys=_split(dyd) if split else None)
    torch.cuda.synchronize()
    assert fused is False  # (the bias gradient is the caller's)
    ref = torch.nn.grad.conv2d_weight(x.double(), (co, ci, 3, 3), dy.double(), padding=1)
    assert rel(dw.double().cpu() - dw0.double(), ref) < CONV_TOL


@pytest.mark.parametrize("silu", [False, True])
def test_winograd_input_gradient_gn_partials(dev, silu):
    """The GroupNorm-backward partials of the dgrad output transform: per channel and 32-pixel block
    {sum dyn, sum dyn * xhat}, dyn = dx * silu'(.) (mvae_conv2d_dgrad_gnbwd_nhwc's contract)."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    n, ci, co, h, w, groups = 2, 128, 64, 8, 16, 32
    g = torch.Generator().manual_seed(11 + silu)
    dy = torch.randn(n, co, h, w, generator=g)
    wt = torch.randn(co, ci, 3, 3, generator=g) / (3 * co ** 0.5)
    xg = torch.randn(n, ci, h, w, generator=g) * 1.5 + 0.3
    gamma, beta = torch.randn(ci, generator=g), torch.randn(ci, generator=g)
    xs = xg.double().reshape(n, groups, -1)
    mean = xs.mean(-1)
    rstd = (xs.var(-1, unbiased=False) + 1e-6).rsqrt()
    link = ops.GnBwdLink(groups, silu)
    link.x, link.gamma, link.beta = cl(xg, dev), gamma.to(dev), beta.to(dev)
    link.mean, link.rstd = mean.float().flatten().to(dev), rstd.float().flatten().to(dev)
    dx = ops.conv2d_dgrad_raw(cl(dy, dev), cl(wt, dev), (n, ci, h, w), ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False),
                              gn_link=link)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_input((n, ci, h, w), wt.double(), dy.double(), padding=1)
    assert rel(dx, ref) < CONV_TOL
    assert link.part is not None and link.dx is dx
    xh = ((xg.double().reshape(n, groups, -1) - mean[..., None]) * rstd[..., None]).reshape(n, ci, h, w)
    d = dx.double().cpu()
    if silu:
        yn = xh * gamma.double()[None, :, None, None] + beta.double()[None, :, None, None]
        sg = torch.sigmoid(yn)
        d = d * sg * (1 + yn * (1 - sg))
    blk = lambda t: t.permute(0, 2, 3, 1).reshape(n * h * w // 32, 32, ci).sum(1)  # noqa: E731
    want = torch.stack([blk(d), blk(d * xh)], -1).flatten()
    assert rel(link.part, want) < 1e-5


def test_winograd_through_conv2d_matches_implicit_gemm(dev, monkeypatch):
    """ops.conv2d forward + backward (dx, dW, db) on the Winograd path against the same layer on the implicit GEMM."""
    from medvae_disentangled_multimodal_amd import ops
    n, c, h, w = 4, 256, 16, 16
    g = torch.Generator().manual_seed(5)
    x0 = torch.randn(n, c, h, w, generator=g)
    w0 = torch.randn(c, c, 3, 3, generator=g) / (3 * c ** 0.5)
    b0 = torch.randn(c, generator=g)
    dy0 = torch.randn(n, c, h, w, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)

    def run(wino):
        monkeypatch.setattr(ops, "WINOGRAD", wino)
        x = cl(x0, dev).requires_grad_(True)
        wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        b = b0.to(dev).requires_grad_(True)
        y = ops.conv2d(x, wt, b, geom)
        y.backward(cl(dy0, dev))
        torch.cuda.synchronize()
        return y.detach().cpu(), x.grad.cpu(), wt.grad.cpu(), b.grad.cpu()

    a, r = run(True), run(False)
    for u, v in zip(a, r):
        assert rel(u, v) < CONV_TOL


def test_winograd_rejects_unsupported_geometry(dev):
    """Channel counts % 4, tile sizes 2 / 4, and fused statistics only on the 32-pixel-block geometries."""
    from medvae_disentangled_multimodal_amd import _lib
    x = torch.zeros(1, 12, 12, 64, device=dev)
    v = torch.zeros(16 * 36 * 64, device=dev)
    with pytest.raises(RuntimeError):
        _lib.call("mvae_winograd_input_transform", x.data_ptr(), v.data_ptr(), 1, 12, 12, 62, 0, 4, 0)
    with pytest.raises(RuntimeError):
        _lib.call("mvae_winograd_input_transform", x.data_ptr(), v.data_ptr(), 1, 12, 12, 64, 0, 3, 0)
    part = torch.zeros(64, device=dev, dtype=torch.float64)
    with pytest.raises(RuntimeError):  # 7x7: no 32-pixel blocks
        _lib.call("mvae_winograd_output_transform", v.data_ptr(), None, None, x.data_ptr(), part.data_ptr(), 1, 7, 7,
                  64, 4, 0)


def test_winograd_kept_input_transform_feeds_weight_gradient(dev, monkeypatch):
    """The forward's V is kept for the weight gradient (WINOGRAD_KEEP_V): one input transform fewer per step, dW bitwise
    equal to the recomputing path."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    n, c, h, w = 2, 128, 16, 16
    g = torch.Generator().manual_seed(9)
    x0 = torch.randn(n, c, h, w, generator=g)
    w0 = torch.randn(c, c, 3, 3, generator=g) / (3 * c ** 0.5)
    dy0 = torch.randn(n, c, h, w, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)

    monkeypatch.setattr(ops, "WINOGRAD_DY2", False)  # (dy's transforms as two kernels: counted below)

    def run(keep):
        monkeypatch.setattr(ops, "WINOGRAD_KEEP_V", keep)
        seen = []
        orig = _lib.call

        def spy(name, *args):
            seen.append(name)
            return orig(name, *args)
        x = cl(x0, dev).requires_grad_(True)
        wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        y = ops.conv2d(x, wt, None, geom)
        monkeypatch.setattr(_lib, "call", spy)
        try:
            y.backward(cl(dy0, dev))
        finally:
            monkeypatch.setattr(_lib, "call", orig)
        torch.cuda.synchronize()
        return x.grad.cpu(), wt.grad.cpu(), seen.count("mvae_winograd_input_transform")

    dxk, dwk, nk = run(True)
    dxr, dwr, nr = run(False)
    assert (nk, nr) == (1, 2)  # backward: dy's transform only, vs dy's and x's
    assert torch.equal(dwk, dwr) and torch.equal(dxk, dxr)



@pytest.mark.parametrize("n,ci,co,h,w", CASES)
@pytest.mark.parametrize("dy_split", [False, True])
def test_winograd_dy_transforms_match_the_two_passes(dev, n, ci, co, h, w, dy_split, _wino_on):
    """mvae_winograd_dy_transforms (one pass over dy) writes exactly what the input gradient's input transform and the
    weight gradient's dy transform write (bitwise: the same operation order)."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    mt = _wino_on
    g = torch.Generator().manual_seed(n * 131 + h * 7 + w)
    dy = cl(torch.randn(n, co, h, w, generator=g), dev)
    src = _split(dy) if dy_split else dy
    t = n * -(-h // mt) * -(-w // mt)
    nbytes = 4 * (mt + 2) ** 2 * t * co
    v1, d1, v2, d2 = (torch.full((nbytes,), 7, dtype=torch.uint8, device=dev) for _ in range(4))
    st = ops._stream(dy)
    _lib.call("mvae_winograd_dy_transforms", src.data_ptr(), v1.data_ptr(), d1.data_ptr(), n, h, w, co,
              int(dy_split), mt, st)
    _lib.call("mvae_winograd_input_transform", src.data_ptr(), v2.data_ptr(), n, h, w, co, int(dy_split), mt, st)
    _lib.call("mvae_winograd_dy_transform", src.data_ptr(), d2.data_ptr(), n, h, w, co, int(dy_split), mt, st)
    torch.cuda.synchronize()
    assert torch.equal(v1, v2) and torch.equal(d1, d2)


def test_winograd_backward_one_pass_over_dy(dev, monkeypatch):
    """Through Conv2dFn's backward: the input gradient's pass over dy keeps D' for the weight gradient (WINOGRAD_DY2):
    one dy kernel instead of two, dx and dW bitwise equal to the two-pass backward."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    n, c, h, w = 2, 128, 16, 16
    g = torch.Generator().manual_seed(11)
    x0 = torch.randn(n, c, h, w, generator=g)
    w0 = torch.randn(c, c, 3, 3, generator=g) / (3 * c ** 0.5)
    dy0 = torch.randn(n, c, h, w, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)

    def run(dy2):
        monkeypatch.setattr(ops, "WINOGRAD_DY2", dy2)
        seen = []
        orig = _lib.call

        def spy(name, *args):
            seen.append(name)
            return orig(name, *args)
        x = cl(x0, dev).requires_grad_(True)
        wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        y = ops.conv2d(x, wt, None, geom)
        monkeypatch.setattr(_lib, "call", spy)
        try:
            y.backward(cl(dy0, dev))
        finally:
            monkeypatch.setattr(_lib, "call", orig)
        torch.cuda.synchronize()
        return x.grad.cpu(), wt.grad.cpu(), [seen.count(k) for k in (
            "mvae_winograd_dy_transforms", "mvae_winograd_dy_transform", "mvae_winograd_input_transform")]

    dx1, dw1, n1 = run(True)
    dx2, dw2, n2 = run(False)
    assert n1 == [1, 0, 0] and n2 == [0, 1, 1]
    assert torch.equal(dx1, dx2) and torch.equal(dw1, dw2)


def _gn_conv_step(dev, x0, g0, b0, w0, cb0, dy0, groups, monkeypatch, **flags):
    """GroupNorm(+SiLU) -> 3x3 conv through ops.group_norm(for_conv=...) and ops.conv2d, forward + backward."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    for k, v in flags.items():
        monkeypatch.setattr(ops, k, v)
    seen = []
    orig = _lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    monkeypatch.setattr(_lib, "call", spy)
    x = cl(x0, dev).requires_grad_(True)
    gam, bet = g0.to(dev).requires_grad_(True), b0.to(dev).requires_grad_(True)
    wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    cb = cb0.to(dev).requires_grad_(True)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)
    h = ops.group_norm(x, gam, bet, groups, 1e-6, silu=True, for_conv=w0.shape[0])
    y = ops.conv2d(h, wt, cb, geom)
    y.backward(cl(dy0, dev))
    torch.cuda.synchronize()
    monkeypatch.setattr(_lib, "call", orig)
    return [t.detach().cpu() for t in (y, x.grad, gam.grad, bet.grad, wt.grad, cb.grad)], seen


@pytest.mark.parametrize("n,c,co,h,w", [(2, 64, 64, 16, 16), (2, 128, 64, 8, 32), (3, 64, 64, 7, 7)])
def test_groupnorm_applied_in_winograd_input_transform(dev, monkeypatch, n, c, co, h, w):
    """GroupNorm+SiLU applied on load by the conv's Winograd input transform (the GroupNorm output never written):
    output and every gradient against float64 autograd, and against the written-output path within 5e-5 (that path
    hands the conv the GroupNorm output pre-split into 3xBF16 hi + lo, 2^-17 from the fp32 value, which the F4
    transform amplifies ~10x)."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(n * c + h)
    x0 = torch.randn(n, c, h, w, generator=g) * 1.3 + 0.2
    g0, b0 = torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1
    w0 = torch.randn(co, c, 3, 3, generator=g) / (3 * c ** 0.5)
    cb0 = torch.randn(co, generator=g)
    dy0 = torch.randn(n, co, h, w, generator=g)
    fused, seen = _gn_conv_step(dev, x0, g0, b0, w0, cb0, dy0, 32, monkeypatch, WINOGRAD_GN=True)
    assert "mvae_winograd_input_transform_gn" in seen and "mvae_group_norm_stats_nhwc" in seen
    assert "mvae_group_norm_apply_nhwc" not in seen and "mvae_group_norm_fwd_nhwc" not in seen
    plain, seen2 = _gn_conv_step(dev, x0, g0, b0, w0, cb0, dy0, 32, monkeypatch, WINOGRAD_GN=False)
    assert "mvae_winograd_input_transform_gn" not in seen2
    for a, b in zip(fused, plain):
        assert rel(a, b) < 5e-5
    xr = x0.double().requires_grad_()
    gr, br = g0.double().requires_grad_(), b0.double().requires_grad_()
    wr, cbr = w0.double().requires_grad_(), cb0.double().requires_grad_()
    yr = F.conv2d(F.silu(F.group_norm(xr, 32, gr, br, eps=1e-6)), wr, cbr, padding=1)
    yr.backward(dy0.double())
    for a, b in zip(fused, (yr, xr.grad, gr.grad, br.grad, wr.grad, cbr.grad)):
        assert rel(a, b) < CONV_TOL


def test_deferred_groupnorm_output_is_written_when_the_conv_cannot_apply_it(dev, monkeypatch):
    """A deferred GroupNorm output whose conv turns out not to run Winograd (here: switched off between the two
    calls) is materialized by mvae_group_norm_apply_nhwc and the implicit GEMM runs on it."""
    import torch.nn.functional as F
    from medvae_disentangled_multimodal_amd import _lib, ops
    n, c, co, h, w = 2, 64, 64, 16, 16
    g = torch.Generator().manual_seed(3)
    x0 = torch.randn(n, c, h, w, generator=g)
    g0, b0 = torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1
    w0 = torch.randn(co, c, 3, 3, generator=g) / (3 * c ** 0.5)
    monkeypatch.setattr(ops, "WINOGRAD_GN", True)
    x = cl(x0, dev).requires_grad_(True)
    gam, bet = g0.to(dev).requires_grad_(True), b0.to(dev).requires_grad_(True)
    wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    hgn = ops.group_norm(x, gam, bet, 32, 1e-6, silu=True, for_conv=co)
    assert getattr(hgn, ops.GN_LAZY_ATTR, None) is not None
    monkeypatch.setattr(ops, "WINOGRAD", False)
    seen = []
    orig = _lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    monkeypatch.setattr(_lib, "call", spy)
    y = ops.conv2d(hgn, wt, None, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False))
    y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    monkeypatch.setattr(_lib, "call", orig)
    assert "mvae_group_norm_apply_nhwc" in seen and "mvae_winograd_gemm" not in seen
    xr, gr, br, wr = (t.double().requires_grad_() for t in (x0, g0, b0, w0))
    yr = F.conv2d(F.silu(F.group_norm(xr, 32, gr, br, eps=1e-6)), wr, None, padding=1)
    yr.backward(torch.ones_like(yr))
    for a, b in ((y, yr), (x.grad, xr.grad), (wt.grad, wr.grad), (gam.grad, gr.grad)):
        assert rel(a, b) < CONV_TOL


def test_winograd_image_chunks(dev, monkeypatch, _wino_on):
    """A batch whose transformed operands exceed one buffer descriptor runs in image chunks (here forced by a small
    limit: 5 images in chunks of 2 / 2 / 1): forward with bias, residual and statistics, input gradient, and the weight
    gradient accumulated over the chunks from the kept per-chunk transforms, against float64."""
    import torch.nn.functional as F
    from medvae_disentangled_multimodal_amd import ops
    n, c, co, h, w = 5, 64, 32, 8, 16
    per_img = (_wino_on + 2) ** 2 * ops._wino_tiles(1, h, w) * c * 4
    monkeypatch.setattr(ops, "_MAX_DESC_BYTES", 2 * per_img)
    assert ops._wino_chunks(n, h, w, c) == [(0, 2), (2, 4), (4, 5)]
    g = torch.Generator().manual_seed(21)
    x0 = torch.randn(n, c, h, w, generator=g)
    w0 = torch.randn(co, c, 3, 3, generator=g) / (3 * c ** 0.5)
    b0 = torch.randn(co, generator=g)
    r0 = torch.randn(n, co, h, w, generator=g)
    dy0 = torch.randn(n, co, h, w, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)
    x = cl(x0, dev).requires_grad_(True)
    wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    b = b0.to(dev).requires_grad_(True)
    y = ops.conv2d(x, wt, b, geom, residual=cl(r0, dev), gn_stats=True)
    part = getattr(y, ops.GN_PART_ATTR)[0]
    y.backward(cl(dy0, dev))
    torch.cuda.synchronize()
    xr, wr, br = (t.double().requires_grad_() for t in (x0, w0, b0))
    yr = F.conv2d(xr, wr, br, padding=1) + r0.double()
    yr.backward(dy0.double())
    assert rel(y, yr) < CONV_TOL
    assert rel(part, _stats64(y.detach().double().cpu())) < 1e-9
    for a, ref in ((x.grad, xr.grad), (wt.grad, wr.grad), (b.grad, br.grad)):
        assert rel(a, ref) < CONV_TOL


def _deferred_gn(dev, monkeypatch, n=2, c=64, co=64, h=16, w=16, seed=4):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(seed)
    x0 = torch.randn(n, c, h, w, generator=g)
    g0, b0 = torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1
    w0 = torch.randn(co, c, 3, 3, generator=g) / (3 * c ** 0.5)
    dy0 = torch.randn(n, co, h, w, generator=g)
    monkeypatch.setattr(ops, "WINOGRAD_GN", True)
    x = cl(x0, dev).requires_grad_(True)
    gam, bet = g0.to(dev).requires_grad_(True), b0.to(dev).requires_grad_(True)
    wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    hgn = ops.group_norm(x, gam, bet, 32, 1e-6, silu=True, for_conv=co)
    assert isinstance(hgn, ops.DeferredGnOutput) and getattr(hgn, ops.GN_LAZY_ATTR, None) is not None
    return (x0, g0, b0, w0, dy0), (x, gam, bet, wt, hgn)


def _ref_grads(x0, g0, b0, w0, dy0):
    import torch.nn.functional as F
    xr, gr, br, wr = (t.double().requires_grad_() for t in (x0, g0, b0, w0))
    yr = F.conv2d(F.silu(F.group_norm(xr, 32, gr, br, eps=1e-6)), wr, None, padding=1)
    yr.backward(dy0.double())
    return yr, xr.grad, gr.grad, wr.grad


def test_deferred_groupnorm_output_refuses_reads(dev, monkeypatch, _wino_on):
    """The deferred placeholder is not the GroupNorm's values: any torch op on it raises (a forward hook or user code
    reading a Normalize output), metadata queries pass, and the consuming conv still runs on it."""
    from medvae_disentangled_multimodal_amd import ops
    _, (x, gam, bet, wt, hgn) = _deferred_gn(dev, monkeypatch)
    assert tuple(hgn.shape) == tuple(x.shape) and hgn.device == x.device and hgn.dtype == torch.float32
    for read in (lambda t: t.sum(), lambda t: t + 1, lambda t: t.clone(), lambda t: t.cpu(), lambda t: float(t[0, 0, 0, 0]),
                 lambda t: torch.nn.functional.relu(t), repr):
        with pytest.raises(RuntimeError, match="deferred"):
            read(hgn)
    y = ops.conv2d(hgn, wt, None, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False))
    assert not isinstance(y, ops.DeferredGnOutput) and torch.isfinite(y).all()


def test_deferred_groupnorm_conv_second_backward(dev, monkeypatch, _wino_on):
    """retain_graph: the second backward through a deferred-GroupNorm Winograd conv (whose kept V the first one released)
    re-derives V from the GroupNorm input and gives the same gradients again."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    (x0, g0, b0, w0, dy0), (x, gam, bet, wt, hgn) = _deferred_gn(dev, monkeypatch)
    y = ops.conv2d(hgn, wt, None, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False))
    dy = cl(dy0, dev)
    y.backward(dy, retain_graph=True)
    torch.cuda.synchronize()
    first = [t.grad.clone() for t in (x, gam, wt)]
    for t in (x, gam, bet, wt):
        t.grad = None
    seen = []
    orig = _lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    monkeypatch.setattr(_lib, "call", spy)
    y.backward(dy)
    torch.cuda.synchronize()
    monkeypatch.setattr(_lib, "call", orig)
    assert "mvae_winograd_input_transform_gn" in seen  # V re-derived, normalized on load
    for a, b in zip((x.grad, gam.grad, wt.grad), first):
        assert rel(a, b) < 1e-6
    yr, xg, gg, wg = _ref_grads(x0, g0, b0, w0, dy0)
    for a, b in ((y, yr), (x.grad, xg), (gam.grad, gg), (wt.grad, wg)):
        assert rel(a, b) < CONV_TOL


def test_deferred_groupnorm_weight_gradient_off_winograd(dev, monkeypatch, _wino_on):
    """The Winograd weight gradient switched off between forward and backward: the weight gradient writes the
    GroupNorm output (mvae_group_norm_apply_nhwc) and runs the implicit GEMM on it -- never on the placeholder."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    (x0, g0, b0, w0, dy0), (x, gam, bet, wt, hgn) = _deferred_gn(dev, monkeypatch)
    y = ops.conv2d(hgn, wt, None, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False))
    monkeypatch.setattr(ops, "WINOGRAD_WGRAD", False)
    seen = []
    orig = _lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    monkeypatch.setattr(_lib, "call", spy)
    y.backward(cl(dy0, dev))
    torch.cuda.synchronize()
    monkeypatch.setattr(_lib, "call", orig)
    assert "mvae_group_norm_apply_nhwc" in seen and "mvae_winograd_wgrad_gemm" not in seen
    yr, xg, gg, wg = _ref_grads(x0, g0, b0, w0, dy0)
    for a, b in ((y, yr), (x.grad, xg), (gam.grad, gg), (wt.grad, wg)):
        assert rel(a, b) < CONV_TOL


def test_no_kept_transform_under_no_grad(dev, monkeypatch, _wino_on):
    """Under torch.no_grad (validation) a Winograd conv keeps no input transform for a backward that never comes."""
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(9)
    x = cl(torch.randn(2, 64, 16, 16, generator=g), dev)
    wt = (torch.randn(64, 64, 3, 3, generator=g) / 24).to(dev).contiguous(memory_format=torch.channels_last)
    wt.requires_grad_(True)
    kept = []
    orig = ops._winograd

    def spy(*a, **k):
        kept.append(k.get("keep") if len(a) < 11 else a[10])
        return orig(*a, **k)
    monkeypatch.setattr(ops, "_winograd", spy)
    with torch.no_grad():
        ops.conv2d(x, wt, None, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False))
    assert kept and all(k is None for k in kept)
    ops.conv2d(x, wt, None, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False))
    assert kept[-1] is not None


ARITH_CASES = [(2, 64, 64, 8, 8), (3, 128, 64, 16, 16), (2, 64, 32, 8, 32), (3, 64, 64, 7, 7), (1, 32, 64, 12, 64),
               (2, 512, 256, 8, 8)]


def _conv_fwd_bwd(dev, x0, w0, b0, dy0, prec, monkeypatch, r0=None):
    """ops.conv2d forward (+ bias, + residual) and backward in arithmetic `prec`, recording the library calls."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    seen = []
    orig = _lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    x = cl(x0, dev).requires_grad_(True)
    wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    b = b0.to(dev).requires_grad_(True)
    monkeypatch.setattr(_lib, "call", spy)
    prev = ops.set_precision(prec)
    try:
        y = ops.conv2d(x, wt, b, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False),
                       residual=cl(r0, dev) if r0 is not None else None)
        y.backward(cl(dy0, dev))
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(prev)
        monkeypatch.setattr(_lib, "call", orig)
    assert {"mvae_winograd_gemm", "mvae_winograd_wgrad_gemm", "mvae_winograd_wgrad_output"} <= set(seen)
    assert "mvae_conv2d_nhwc" not in seen and "mvae_conv2d_wgrad_nhwc" not in seen
    return y.detach().cpu(), x.grad.cpu(), wt.grad.cpu(), b.grad.cpu()


@pytest.mark.parametrize("n,ci,co,h,w", ARITH_CASES)
def test_winograd_exact_fp32(dev, n, ci, co, h, w, monkeypatch, _wino_on):
    """The exact-fp32 arithmetic ("32-exact", the c4x line) on the Winograd form: V / U / D' written as a bit split the
    f32-input MFMA reassembles exactly, so the result differs from float64 only by the transforms' fp32 rounding
    (simulated: F(4x4) ~5e-7, F(2x2) ~8e-8; the direct fp32 conv ~4e-8). Forward with bias and residual, input gradient,
    weight gradient and bias gradient against float64 at 5e-6 -- 40x inside the 3xBF16 bar."""
    import torch.nn.functional as F
    g = torch.Generator().manual_seed(n * ci + co + 7 * h + w)
    x0 = torch.randn(n, ci, h, w, generator=g)
    w0 = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
    b0, r0 = torch.randn(co, generator=g), torch.randn(n, co, h, w, generator=g)
    dy0 = torch.randn(n, co, h, w, generator=g)
    y, dx, dw, db = _conv_fwd_bwd(dev, x0, w0, b0, dy0, "32-exact", monkeypatch, r0)
    xr, wr, br = (t.double().requires_grad_() for t in (x0, w0, b0))
    yr = F.conv2d(xr, wr, br, padding=1) + r0.double()
    yr.backward(dy0.double())
    for a, ref in ((y, yr), (dx, xr.grad), (dw, wr.grad), (db, br.grad)):
        assert rel(a, ref) < 5e-6


# (cout 32 with 32 / 64 input channels takes the direct cout-32 weight-gradient kernel outside the exact mode: 48 here)
BF16_CASES = [c if c[2] != 32 else (c[0], c[1], 48, c[3], c[4]) for c in ARITH_CASES]


@pytest.mark.parametrize("n,ci,co,h,w", BF16_CASES)
def test_winograd_bf16_matches_emulation(dev, n, ci, co, h, w, monkeypatch, _wino_on):
    """The bf16-mixed arithmetic on the Winograd form (c5): the GEMM multiplies V, U (and D') rounded to bf16 in the
    transform domain, so it is checked against the float64 emulation of exactly that algorithm (tests/wino_ref.py:
    the same transforms, the GEMM operands rounded to bf16 RNE) -- and against the float64 conv at the algorithm's own
    bf16 error (m = 2 ~4e-3, m = 4 ~3e-2). Against the emulation only fp32 accumulation and the transforms' fp32
    rounding differ; the latter flips the bf16 rounding of a few transform-domain elements whose float64 value lies
    within ~1e-7 of a rounding boundary, each a 2^-8 change amplified by the output transform (A^T up to 8 at m = 4):
    measured up to 4e-4 at m = 4, 3e-5 at m = 2 -- bars 1e-3 / 2e-4."""
    import torch.nn.functional as F
    import wino_ref as W
    from medvae_disentangled_multimodal_amd import ops
    monkeypatch.setattr(ops, "WINOGRAD_TILE_BF16", _wino_on)
    monkeypatch.setattr(ops, "WINOGRAD_BF16_MAX_W", 64)
    g = torch.Generator().manual_seed(n * ci + co + 5 * h + w)
    x0 = torch.randn(n, ci, h, w, generator=g)
    w0 = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
    b0 = torch.randn(co, generator=g)
    dy0 = torch.randn(n, co, h, w, generator=g)
    y, dx, dw, db = _conv_fwd_bwd(dev, x0, w0, b0, dy0, "bf16-mixed", monkeypatch)
    m = _wino_on
    ye = W.conv(x0, w0, m, W.bf16) + b0.double().view(1, -1, 1, 1)
    dxe = W.conv(dy0, W.dgrad_weights(w0), m, W.bf16)
    dwe = W.wgrad(x0, dy0, m, W.bf16)
    errs = {k: rel(a, ref) for k, a, ref in (("y", y, ye), ("dx", dx, dxe), ("dw", dw, dwe))}
    assert all(v < (2e-4 if m == 2 else 1e-3) for v in errs.values()), errs
    assert rel(db, dy0.double().sum((0, 2, 3))) < 1e-5
    xr, wr = x0.double().requires_grad_(), w0.double().requires_grad_()
    yr = F.conv2d(xr, wr, b0.double(), padding=1)
    yr.backward(dy0.double())
    bar = 1e-2 if m == 2 else 6e-2
    errs = {k: rel(a, ref) for k, a, ref in (("y", y, yr), ("dx", dx, xr.grad), ("dw", dw, wr.grad))}
    assert all(v < bar for v in errs.values()), errs


def test_winograd_exact_fp32_groupnorm_on_load_and_chunks(dev, monkeypatch, _wino_on):
    """The exact arithmetic through the GroupNorm-on-load transform and over image chunks (5 images in chunks of
    2 / 2 / 1 under a small descriptor limit): every gradient against float64 at 5e-6."""
    import torch.nn.functional as F
    from medvae_disentangled_multimodal_amd import ops
    n, c, co, h, w = 5, 64, 64, 8, 16
    per_img = (_wino_on + 2) ** 2 * ops._wino_tiles(1, h, w) * c * 4
    monkeypatch.setattr(ops, "_MAX_DESC_BYTES", 2 * per_img)
    g = torch.Generator().manual_seed(77)
    x0 = torch.randn(n, c, h, w, generator=g) * 1.3 + 0.2
    g0, b0 = torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1
    w0 = torch.randn(co, c, 3, 3, generator=g) / (3 * c ** 0.5)
    cb0 = torch.randn(co, generator=g)
    dy0 = torch.randn(n, co, h, w, generator=g)
    prev = ops.set_precision("32-exact")
    try:
        fused, seen = _gn_conv_step(dev, x0, g0, b0, w0, cb0, dy0, 32, monkeypatch, WINOGRAD_GN=True)
    finally:
        ops.restore_math_mode(prev)
    assert seen.count("mvae_winograd_input_transform_gn") == 3 and "mvae_group_norm_apply_nhwc" not in seen
    xr = x0.double().requires_grad_()
    gr, br = g0.double().requires_grad_(), b0.double().requires_grad_()
    wr, cbr = w0.double().requires_grad_(), cb0.double().requires_grad_()
    yr = F.conv2d(F.silu(F.group_norm(xr, 32, gr, br, eps=1e-6)), wr, cbr, padding=1)
    yr.backward(dy0.double())
    for a, b in zip(fused, (yr, xr.grad, gr.grad, br.grad, wr.grad, cbr.grad)):
        assert rel(a, b) < 5e-6


def test_winograd_exact_rejects_split_inputs(dev):
    """A pre-split input is a 3xBF16 value split; the exact mode's transforms refuse one instead of reading it as bits."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    x = torch.zeros(1, 8, 8, 8, device=dev).contiguous(memory_format=torch.channels_last)
    v = torch.empty(36 * 4 * 8 * 4, dtype=torch.uint8, device=dev)
    prev = ops.set_precision("32-exact")
    try:
        with pytest.raises(RuntimeError, match="exact"):
            _lib.call("mvae_winograd_input_transform", x.data_ptr(), v.data_ptr(), 1, 8, 8, 8, 1, 4, ops._stream(x))
    finally:
        ops.restore_math_mode(prev)


def test_deferred_groupnorm_conv_at_32_channels(dev, monkeypatch, _wino_on):
    """A deferred GroupNorm (one channel per group) feeding a 32 -> 32 Winograd conv: its weight gradient must be the
    Winograd one on the kept V -- the direct cout-32 weight-gradient kernel, which the dispatcher otherwise picks for
    32-channel convs, would read the placeholder as x (an out-of-bounds read of a one-element allocation)."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    (x0, g0, b0, w0, dy0), (x, gam, bet, wt, hgn) = _deferred_gn(dev, monkeypatch, n=2, c=32, co=32, h=16, w=16)
    seen = []
    orig = _lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    monkeypatch.setattr(_lib, "call", spy)
    y = ops.conv2d(hgn, wt, None, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False))
    y.backward(cl(dy0, dev))
    torch.cuda.synchronize()
    monkeypatch.setattr(_lib, "call", orig)
    assert "mvae_winograd_wgrad_gemm" in seen and "mvae_conv2d_wgrad_direct_nhwc" not in seen
    yr, xg, gg, wg = _ref_grads(x0, g0, b0, w0, dy0)
    for a, b in ((y, yr), (x.grad, xg), (gam.grad, gg), (wt.grad, wg)):
        assert rel(a, b) < CONV_TOL


def _conv_gn_conv(dev, monkeypatch, link_on, x0, wa0, ba0, g0, b0, wb0, dy0, prec="32"):
    """conv A (GroupNorm statistics from its epilogue) -> GroupNorm(32)+SiLU deferred -> conv B: the ResnetBlock's
    conv1 -> norm2 -> conv2 edge, with the GroupNorm backward's partials from conv B's Winograd input gradient (link_on)
    or from its own pass, and conv A's dy pre-split by the GroupNorm backward (DySplit) either way."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    monkeypatch.setattr(ops, "WINOGRAD_GN", True)
    monkeypatch.setattr(ops, "WINOGRAD_GN_LINK", link_on)
    monkeypatch.setattr(ops, "DYSPLIT_MIN_MACS", 0.0)
    seen = []
    orig = _lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    x = cl(x0, dev).requires_grad_(True)
    wa = wa0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    ba = ba0.to(dev).requires_grad_(True)
    gam, bet = g0.to(dev).requires_grad_(True), b0.to(dev).requires_grad_(True)
    wb = wb0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)
    orig_path = _lib.call("mvae_set_group_norm_path", 1)  # (the streaming GroupNorm chain at this test size)
    pv = ops.set_precision(prec)
    monkeypatch.setattr(_lib, "call", spy)
    try:
        h = ops.conv2d(x, wa, ba, geom, gn_stats=True)
        hg = ops.group_norm(h, gam, bet, 32, 1e-6, silu=True, for_conv=wb0.shape[0])
        y = ops.conv2d(hg, wb, None, geom)
        y.backward(cl(dy0, dev))
        torch.cuda.synchronize()
    finally:
        monkeypatch.setattr(_lib, "call", orig)
        _lib.call("mvae_set_group_norm_path", 0)
        ops.restore_math_mode(pv)
    return [t.detach().cpu() for t in (y, x.grad, wa.grad, ba.grad, gam.grad, bet.grad, wb.grad)], seen


@pytest.mark.parametrize("prec,dy_split", [("32", False), ("32", True), ("32-exact", False)])
def test_groupnorm_partials_from_winograd_input_gradient(dev, monkeypatch, _wino_on, prec, dy_split):
    """The deferred GroupNorm's backward takes its partials from the consuming Winograd conv's input-gradient output
    transform (mvae_winograd_output_gnbwd) and still writes the producing conv's dy pre-split with its bias gradient
    (mvae_group_norm_bwd_part_split_nhwc; for a Winograd producer, which splits dy itself, the bias gradient alone;
    the split copy with MVAE_WINOGRAD_DY_SPLIT=1): every output and gradient equals the
    path with the GroupNorm's own partial pass (5e-6: the partials' sums in another order) and float64 (the conv bar)."""
    import torch.nn.functional as F
    n, c, h, w = 2, 128, 16, 16
    g = torch.Generator().manual_seed(31)
    x0 = torch.randn(n, c, h, w, generator=g)
    wa0 = torch.randn(c, c, 3, 3, generator=g) / (3 * c ** 0.5)
    ba0 = torch.randn(c, generator=g) * 0.1
    g0, b0 = torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1
    wb0 = torch.randn(c, c, 3, 3, generator=g) / (3 * c ** 0.5)
    dy0 = torch.randn(n, c, h, w, generator=g)
    from medvae_disentangled_multimodal_amd import ops
    monkeypatch.setattr(ops, "WINOGRAD_DY_FP32", not dy_split)
    linked, seen = _conv_gn_conv(dev, monkeypatch, True, x0, wa0, ba0, g0, b0, wb0, dy0, prec)
    assert "mvae_winograd_output_gnbwd" in seen and "mvae_group_norm_bwd_part_split_nhwc" in seen
    # (a Winograd conv takes dy in fp32: the bias gradient alone; opt-in: the split copy)
    own = "mvae_group_norm_bwd_split_nhwc" if dy_split else "mvae_group_norm_bwd_colsum_nhwc"
    assert own not in seen and "mvae_bias_grad" not in seen
    plain, seen2 = _conv_gn_conv(dev, monkeypatch, False, x0, wa0, ba0, g0, b0, wb0, dy0, prec)
    assert "mvae_winograd_output_gnbwd" not in seen2 and own in seen2
    for a, b in zip(linked, plain):
        assert rel(a, b) < 5e-6
    xr, war, bar_, gr, br, wbr = (t.double().requires_grad_() for t in (x0, wa0, ba0, g0, b0, wb0))
    yr = F.conv2d(F.silu(F.group_norm(F.conv2d(xr, war, bar_, padding=1), 32, gr, br, eps=1e-6)), wbr, None, padding=1)
    yr.backward(dy0.double())
    for a, b in zip(linked, (yr, xr.grad, war.grad, bar_.grad, gr.grad, br.grad, wbr.grad)):
        assert rel(a, b) < CONV_TOL


UPS_CASES = [(2, 64, 64, 8, 8), (2, 32, 64, 16, 16), (1, 64, 32, 12, 8), (2, 128, 64, 4, 32)]


@pytest.mark.parametrize("prec", ["32", "32-exact", "bf16-mixed"])
@pytest.mark.parametrize("n,ci,co,h,w", UPS_CASES)
def test_winograd_upsample_conv(dev, n, ci, co, h, w, prec, monkeypatch, _wino_on):
    """The Upsample conv (nearest x2 + 3x3 / pad 1) as four class convs sharing one Winograd input transform: forward
    with bias, input gradient and weight gradient through ops.conv2d, against float64 (3xBF16 at the conv bar, exact
    fp32 at 5e-6) or, in the bf16 mode, against the float64 emulation of the same algorithm (tests/wino_ref.py)."""
    import torch.nn.functional as F
    import wino_ref as W
    from medvae_disentangled_multimodal_amd import _lib, ops
    monkeypatch.setattr(ops, "WINOGRAD_TILE_BF16", _wino_on)
    monkeypatch.setattr(ops, "WINOGRAD_BF16_MAX_W", 64)
    monkeypatch.setattr(ops, "WINOGRAD_UPSAMPLE_BF16", True)
    g = torch.Generator().manual_seed(n * ci + co + h + w)
    x0 = torch.randn(n, ci, h, w, generator=g)
    w0 = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
    b0 = torch.randn(co, generator=g) * 0.1
    dy0 = torch.randn(n, co, 2 * h, 2 * w, generator=g)
    seen = []
    orig = _lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    x = cl(x0, dev).requires_grad_(True)
    wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    b = b0.to(dev).requires_grad_(True)
    monkeypatch.setattr(_lib, "call", spy)
    pv = ops.set_precision(prec)
    try:
        y = ops.conv2d(x, wt, b, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, True))
        y.backward(cl(dy0, dev))
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(pv)
        monkeypatch.setattr(_lib, "call", orig)
    assert {"mvae_winograd_output_transform_upsample", "mvae_winograd_dy_transforms_upsample",
            "mvae_winograd_upsample_fold"} <= set(seen)
    assert "mvae_conv2d_upsample_nhwc" not in seen and "mvae_conv2d_wgrad_upsample_nhwc" not in seen
    assert tuple(y.shape) == (n, co, 2 * h, 2 * w)
    if prec == "bf16-mixed":
        m = _wino_on
        refs = (W.ups_conv(x0, w0, m, W.bf16) + b0.double().view(1, -1, 1, 1), W.ups_dgrad(dy0, w0, m, W.bf16),
                W.ups_wgrad(x0, dy0, m, W.bf16))
        tol = 2e-4 if m == 2 else 1e-3
    else:
        xr, wr, br = (t.double().requires_grad_() for t in (x0, w0, b0))
        yr = F.conv2d(F.interpolate(xr, scale_factor=2.0, mode="nearest"), wr, br, padding=1)
        yr.backward(dy0.double())
        refs = (yr, xr.grad, wr.grad)
        tol = CONV_TOL if prec == "32" else 5e-6
    errs = {k: rel(a, r) for k, a, r in zip(("y", "dx", "dw"), (y, x.grad, wt.grad), refs)}
    assert all(v < tol for v in errs.values()), errs
    assert rel(b.grad, dy0.double().sum((0, 2, 3))) < 1e-5


def test_winograd_upsample_image_chunks(dev, monkeypatch, _wino_on):
    """The Upsample conv's Winograd form over image chunks (5 images, chunks of 2 / 2 / 1 under a small descriptor
    limit): the class kernels' gradients accumulate over the chunks before the fold."""
    import torch.nn.functional as F
    from medvae_disentangled_multimodal_amd import ops
    n, c, co, h, w = 5, 32, 32, 8, 8
    per_img = (_wino_on + 2) ** 2 * ops._wino_tiles(1, h, w) * 4 * co * 4
    monkeypatch.setattr(ops, "_MAX_DESC_BYTES", 2 * per_img)
    assert ops._wino_chunks(n, h, w, 4 * co) == [(0, 2), (2, 4), (4, 5)]
    g = torch.Generator().manual_seed(8)
    x0 = torch.randn(n, c, h, w, generator=g)
    w0 = torch.randn(co, c, 3, 3, generator=g) / (3 * c ** 0.5)
    dy0 = torch.randn(n, co, 2 * h, 2 * w, generator=g)
    x = cl(x0, dev).requires_grad_(True)
    wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = ops.conv2d(x, wt, None, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, True))
    y.backward(cl(dy0, dev))
    torch.cuda.synchronize()
    xr, wr = x0.double().requires_grad_(), w0.double().requires_grad_()
    yr = F.conv2d(F.interpolate(xr, scale_factor=2.0, mode="nearest"), wr, None, padding=1)
    yr.backward(dy0.double())
    for a, r in ((y, yr), (x.grad, xr.grad), (wt.grad, wr.grad)):
        assert rel(a, r) < CONV_TOL


def _conv_gn_bias(dev, monkeypatch, dybias, prec, ups, gn_path, x0, w0, b0, g0, be0, dy0):
    """conv (3x3 with GroupNorm statistics, or the Upsample conv) -> GroupNorm(32)+SiLU, backward from dy0, with the
    conv's bias gradient from the GroupNorm backward's column sums of dx (dybias) or from its own pass over dy."""
    from medvae_disentangled_multimodal_amd import _lib, ops
    monkeypatch.setattr(ops, "DYBIAS", dybias)
    seen = []
    orig = _lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    x = cl(x0, dev).requires_grad_(True)
    wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    b = b0.to(dev).requires_grad_(True)
    gam, bet = g0.to(dev).requires_grad_(True), be0.to(dev).requires_grad_(True)
    pv = ops.set_precision(prec)
    orig_path = _lib.call("mvae_set_group_norm_path", gn_path)
    monkeypatch.setattr(_lib, "call", spy)
    try:
        h = ops.conv2d(x, wt, b, ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, ups), gn_stats=not ups, gn_bias=ups)
        y = ops.group_norm(h, gam, bet, 32, 1e-6, silu=True)
        y.backward(cl(dy0, dev))
        torch.cuda.synchronize()
    finally:
        monkeypatch.setattr(_lib, "call", orig)
        _lib.call("mvae_set_group_norm_path", 0)
        ops.restore_math_mode(pv)
    del orig_path
    return [t.detach().cpu() for t in (y, x.grad, wt.grad, b.grad, gam.grad, bet.grad)], seen


@pytest.mark.parametrize("prec,ups", [("32-exact", False), ("32-exact", True), ("32", True)])
@pytest.mark.parametrize("gn_path", [0, 1], ids=["auto", "streaming"])
def test_conv_bias_gradient_from_groupnorm_backward(dev, monkeypatch, prec, ups, gn_path, _wino_on):
    """A Winograd conv that reads dy in fp32 (exact fp32; the Upsample conv's Winograd form) and feeds a GroupNorm takes
    its bias gradient from that GroupNorm's backward (mvae_group_norm_bwd_colsum_nhwc: column sums of dx, resident and
    streaming kernels) instead of a column-sum pass over dy: every gradient equals the separate-pass path (bias: fp64
    sums in another order, 1e-6) and float64."""
    import torch.nn.functional as F
    n, c, hw = 2, 64, (8 if ups else 16)
    g = torch.Generator().manual_seed(41 + ups)
    x0 = torch.randn(n, c, hw, hw, generator=g)
    w0 = torch.randn(c, c, 3, 3, generator=g) / (3 * c ** 0.5)
    b0 = torch.randn(c, generator=g) * 0.1
    g0, be0 = torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1
    ho = 2 * hw if ups else hw
    dy0 = torch.randn(n, c, ho, ho, generator=g)
    on, seen = _conv_gn_bias(dev, monkeypatch, True, prec, ups, gn_path, x0, w0, b0, g0, be0, dy0)
    off, seen2 = _conv_gn_bias(dev, monkeypatch, False, prec, ups, gn_path, x0, w0, b0, g0, be0, dy0)
    assert "mvae_group_norm_bwd_colsum_nhwc" in seen and "mvae_group_norm_bwd_colsum_nhwc" not in seen2
    assert ("mvae_winograd_dy_transforms_upsample" if ups else "mvae_winograd_wgrad_gemm") in seen
    for k, (a, b) in enumerate(zip(on, off)):
        assert rel(a, b) < 1e-6, k
    xr, wr, br, gr, bb = (t.double().requires_grad_() for t in (x0, w0, b0, g0, be0))
    xi = F.interpolate(xr, scale_factor=2.0, mode="nearest") if ups else xr
    yr = F.silu(F.group_norm(F.conv2d(xi, wr, br, padding=1), 32, gr, bb, eps=1e-6))
    yr.backward(dy0.double())
    tol = 5e-6 if prec == "32-exact" else CONV_TOL
    for a, b in zip(on, (yr, xr.grad, wr.grad, br.grad, gr.grad, bb.grad)):
        assert rel(a, b) < tol
