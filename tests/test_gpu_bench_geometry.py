"""Hot-path numerics at the bench's own geometry (c4: batch 256, 64x64 input; c2: batch 256, 28x28x3; c3: batch 512,
28x28x3). The GEMM planner picks tiles, split-K factors and the direct weight-gradient path from M = B*H*W, so the
launches the bench times (c4: M = 16,384 at the 8x8x2048 level, 65,536 at 16x16, 1,048,576 for the 32 -> 64 Upsample;
c2: 12,544 at 7x7x512 -- split-K forward / input gradient --, 200,704 at 28x28x128; c3: 401,408 at 28x28x32 -- the
direct cout-32 weight gradient) differ from the small-batch parity cases. Here the hottest convolutions of each config
(3x3, the 1x1 attention / shortcut convs, the stride-2 Downsample with its (0, 1, 0, 1) pad, the Upsample) run at
the bench batch in the default fp32-class (3xBF16) arithmetic -- forward, input gradient and weight gradient through
the same ops.conv2d autograd path the model uses -- and are checked against float64 on a sampled subset: output rows
(pixels x all channels), input-gradient rows, and weight-gradient columns (output channels x all taps / inputs).
Tolerance 2e-4 relative per sampled block (the CONV_TOL of tests/test_gpu_kernels.py).
The two deepest layers (and a 64 x 32x32 x 256 layer with its stride-2 Downsample, 256 tiles of 256x256) also run in the
bf16-mixed arithmetic (config 5; every pass on packed bf16 operands through the LDS-DMA GEMM main loop): the float64
reference then uses the bf16-rounded operands of each GEMM, so only fp32 accumulation differs -- tolerance 1e-4
(sqrt(K) * 2^-24 for K = 18,432 is ~8e-6). The bf16 layers that run the Winograd F(2x2, 3x3) form (c5's 8x8 and
16x16 levels: V, U, D' rounded to bf16 in the transform domain) are checked against the float64 emulation of that
algorithm instead (tests/wino_ref.py), at 2e-4."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
TOL = 2e-4

# n, cin, cout, h, w (input), k, stride, pads (t, l, b, r), upsample
C4 = [(256, 2048, 2048, 8, 8, 3, 1, (1, 1, 1, 1), False), (256, 1024, 1024, 16, 16, 3, 1, (1, 1, 1, 1), False),
      (256, 512, 512, 32, 32, 3, 1, (1, 1, 1, 1), True)]
# the c4 levels the bench runs in Winograd F(4x4, 3x3) form besides the two above: 32x32x512, 64x64x256 and the decoder's
# 64x64 512 -> 256 conv, whose transformed input exceeds one 4 GiB buffer descriptor (two image chunks)
C4W = [(256, 512, 512, 32, 32, 3, 1, (1, 1, 1, 1), False), (256, 256, 256, 64, 64, 3, 1, (1, 1, 1, 1), False),
       (256, 512, 256, 64, 64, 3, 1, (1, 1, 1, 1), False)]
C2 = [(256, 512, 512, 7, 7, 3, 1, (1, 1, 1, 1), False), (256, 512, 512, 7, 7, 1, 1, (0, 0, 0, 0), False),
      (256, 128, 128, 28, 28, 3, 1, (1, 1, 1, 1), False), (256, 128, 128, 28, 28, 3, 2, (0, 0, 1, 1), False),
      (256, 256, 256, 14, 14, 3, 1, (1, 1, 1, 1), True), (256, 512, 256, 7, 7, 3, 1, (1, 1, 1, 1), False)]
C3 = [(512, 32, 32, 28, 28, 3, 1, (1, 1, 1, 1), False), (512, 64, 64, 14, 14, 3, 1, (1, 1, 1, 1), False),
      (512, 128, 128, 7, 7, 3, 1, (1, 1, 1, 1), False), (512, 128, 128, 7, 7, 1, 1, (0, 0, 0, 0), False),
      (512, 32, 32, 28, 28, 3, 2, (0, 0, 1, 1), False), (512, 64, 64, 14, 14, 3, 1, (1, 1, 1, 1), True)]
# bf16-mixed (config 5): the c4 layers above plus a 64 x 32x32 x 256 layer (fwd M = 65,536: 256 tiles of 256x256) and
# its stride-2 Downsample, every pass on the LDS-DMA main loop
C5 = C4[:2] + [(64, 256, 256, 32, 32, 3, 1, (1, 1, 1, 1), False), (64, 256, 256, 64, 64, 3, 2, (0, 0, 1, 1), False)]
LAYERS = [("c4", l, "32") for l in C4 + C4W] + [("c5", l, "bf16-mixed") for l in C5] + \
    [("c2", l, "32") for l in C2] + [("c3", l, "32") for l in C3]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _src(o, r, stride, pad, size, ups):
    """input index feeding output o through tap r (stride, leading pad, optional nearest x2 upsample), or -1."""
    u = o * stride - pad + r
    lim = 2 * size if ups else size
    ok = (u >= 0) & (u < lim)
    s = torch.div(u, 2, rounding_mode="floor") if ups else u
    return torch.where(ok, s, torch.full_like(s, -1))


def _gather(x, n, ih, iw):
    """x [N, C, H, W] -> rows [len, C] at (n, ih, iw), zeros where ih or iw is -1."""
    ok = (ih >= 0) & (iw >= 0)
    v = x[n, :, ih.clamp_min(0), iw.clamp_min(0)]
    return v * ok[:, None].to(v.dtype)


def _rel(a, b):
    return float((a.double() - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.parametrize("cfg,layer,prec", LAYERS, ids=lambda v: str(v).replace(" ", ""))
def test_hot_conv_at_bench_batch(dev, cfg, layer, prec):
    from medvae_disentangled_multimodal_amd import ops
    n, ci, co, h, w, k, st, (pt, pl, pb, pr), ups = layer
    tol = TOL if prec == "32" else 1e-4
    g = torch.Generator().manual_seed(ci + h + 7 * k + st)
    x = torch.randn(n, ci, h, w, generator=g)
    wt = torch.randn(co, ci, k, k, generator=g) / math.sqrt(ci * k * k)
    b = torch.randn(co, generator=g) * 0.1
    geom = ops.ConvGeom(k, k, st, pt, pl, pb, pr, ups)
    ho, wo = geom.out_hw(h, w)
    xd = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    wd = wt.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    bd = b.to(dev).requires_grad_()
    dy = torch.randn(n, co, ho, wo, generator=g)
    seen = []
    orig = ops._lib.call

    def spy(name, *args):
        seen.append(name)
        return orig(name, *args)
    prev = ops.set_precision(prec)
    try:
        wino = ops._wino_ok(geom, n, h, w, ci, co)
        mt = ops._wtile()
        ops._lib.call = spy
        y = ops.conv2d(xd, wd, bd, geom)
        y.backward(dy.to(dev).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
    finally:
        ops._lib.call = orig
        ops.restore_math_mode(prev)
    assert ops._lib.query("mvae_get_math_mode") == 0
    assert tuple(y.shape) == (n, co, ho, wo)
    if (cfg, layer) in [("c4", l) for l in C4W]:
        assert wino  # (these are the layers the bench times on the Winograd form)
    if wino:  # forward, input gradient and weight gradient all on the Winograd entry points
        assert seen.count("mvae_winograd_gemm") >= 2 and seen.count("mvae_winograd_wgrad_gemm") >= 1
        assert "mvae_winograd_output_transform" in seen and "mvae_winograd_wgrad_output" in seen
        assert "mvae_conv2d_nhwc" not in seen and "mvae_conv2d_wgrad_nhwc" not in seen
        chunks = ops._wino_chunks(n, h, w, max(ci, co))
        if (h, ci) == (64, 512):  # the real 4 GiB descriptor limit splits this one, at the bench batch
            assert len(chunks) == 2 and seen.count("mvae_winograd_wgrad_gemm") == 2

    if prec != "32" and wino:
        # bf16 on the Winograd form (c5's 8x8 / 16x16 levels): the GEMM multiplies V, U, D' rounded to bf16 in the
        # transform domain -- checked against the float64 emulation of that algorithm (tests/wino_ref.py) on the same
        # sampled blocks; only fp32 accumulation and the transforms' fp32 rounding differ
        import wino_ref as W
        ns = torch.randint(0, n, (96,), generator=g)
        oh, ow = torch.randint(0, ho, (96,), generator=g), torch.randint(0, wo, (96,), generator=g)
        got = y.detach()[ns.to(dev), :, oh.to(dev), ow.to(dev)].cpu()
        assert _rel(got, W.rows(x, wt, b, ns, oh, ow, mt, W.bf16)) < 2e-4
        ih, iw = torch.randint(0, h, (96,), generator=g), torch.randint(0, w, (96,), generator=g)
        got = xd.grad[ns.to(dev), :, ih.to(dev), iw.to(dev)].cpu()
        assert _rel(got, W.rows(dy, W.dgrad_weights(wt), None, ns, ih, iw, mt, W.bf16)) < 2e-4
        cols = torch.randperm(co, generator=g)[:4]
        assert _rel(wd.grad[cols.to(dev)].cpu(), W.wgrad(x, dy, mt, W.bf16, cols=cols)) < 2e-4
        assert _rel(bd.grad.cpu(), dy.double().sum((0, 2, 3))) < 1e-5
        return
    if prec == "32":
        xs, ws, dys = x.double(), wt.double(), dy.double()
    else:
        xs, ws, dys = x.bfloat16().double(), wt.bfloat16().double(), dy.bfloat16().double()
    ns = torch.randint(0, n, (96,), generator=g)
    # forward rows: y[n, :, oh, ow] = sum_{r,s} W[:, :, r, s] x_src(n, oh, ow, r, s) + b
    oh, ow = torch.randint(0, ho, (96,), generator=g), torch.randint(0, wo, (96,), generator=g)
    ref = b.double()[None, :].repeat(96, 1)
    for r in range(k):
        for s in range(k):
            ref += _gather(xs, ns, _src(oh, r, st, pt, h, ups), _src(ow, s, st, pl, w, ups)) @ ws[:, :, r, s].t()
    got = y.detach()[ns.to(dev), :, oh.to(dev), ow.to(dev)].cpu()
    assert _rel(got, ref) < tol
    # input-gradient rows: dx[n, :, ih, iw] = sum over (upsampled copy a, c) and taps of dy at the output it fed
    ih, iw = torch.randint(0, h, (96,), generator=g), torch.randint(0, w, (96,), generator=g)
    ref = torch.zeros(96, ci, dtype=torch.float64)
    copies = (0, 1) if ups else (0,)
    for a in copies:
        for c in copies:
            uh, uw = (2 * ih + a, 2 * iw + c) if ups else (ih, iw)
            for r in range(k):
                for s in range(k):
                    nh, nw = uh + pt - r, uw + pl - s
                    o_h, o_w = torch.div(nh, st, rounding_mode="floor"), torch.div(nw, st, rounding_mode="floor")
                    ok = (nh >= 0) & (nw >= 0) & (nh % st == 0) & (nw % st == 0) & (o_h < ho) & (o_w < wo)
                    v = dys[ns, :, o_h.clamp(0, ho - 1), o_w.clamp(0, wo - 1)] * ok[:, None].double()
                    ref += v @ ws[:, :, r, s]
    got = xd.grad[ns.to(dev), :, ih.to(dev), iw.to(dev)].cpu()
    assert _rel(got, ref) < tol
    # weight-gradient columns: dW[o, :, r, s] = sum over all n, oh, ow of dy[n, o, oh, ow] x_src(n, oh, ow, r, s)
    cols = torch.randperm(co, generator=g)[:4]
    ref = torch.zeros(4, ci, k, k, dtype=torch.float64)
    xin = F.interpolate(xs, scale_factor=2.0, mode="nearest") if ups else xs
    for n0 in range(0, n, 32):
        xp = F.pad(xin[n0:n0 + 32], (pl, pr, pt, pb))
        d = dys[n0:n0 + 32][:, cols]  # [32, 4, ho, wo]
        for r in range(k):
            for s in range(k):
                xt = xp[:, :, r:r + st * (ho - 1) + 1:st, s:s + st * (wo - 1) + 1:st]
                ref[:, :, r, s] += torch.einsum("nohw,nchw->oc", d, xt)
    got = wd.grad[cols.to(dev)].cpu()
    assert _rel(got, ref) < tol
    assert _rel(bd.grad.cpu(), dy.double().sum((0, 2, 3))) < 1e-5


@pytest.mark.parametrize("ci,co", [(256, 256), (512, 256)], ids=["64x64x256", "64x64x512-256-chunked"])
def test_groupnorm_on_load_winograd_conv_at_bench_batch(dev, ci, co, monkeypatch):
    """c4's GroupNorm(32)+SiLU -> 3x3 conv edge at 64x64 and B = 256, as the bench runs it: the GroupNorm computes its
    statistics only, the conv's Winograd input transform normalizes on load (the GroupNorm output is never written),
    the weight gradient reads the kept transform (512 -> 256: per image chunk). Checked against float64: output rows and
    weight-gradient columns on sampled blocks, and the whole input / gamma gradient of two sampled images (GroupNorm and
    conv are per image, so one image's autograd in float64 is exact); against the written-output path (the GroupNorm
    writing its output, pre-split) within 5e-5 over the whole tensors."""
    from medvae_disentangled_multimodal_amd import ops
    n, h, w = 256, 64, 64
    g = torch.Generator().manual_seed(ci + co)
    x0 = torch.randn(n, ci, h, w, generator=g) * 1.3 + 0.2
    g0, b0 = torch.rand(ci, generator=g) + 0.5, torch.randn(ci, generator=g) * 0.1
    w0 = torch.randn(co, ci, 3, 3, generator=g) / (3 * ci ** 0.5)
    cb0 = torch.randn(co, generator=g) * 0.1
    dy0 = torch.randn(n, co, h, w, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)

    def run(lazy_on):
        monkeypatch.setattr(ops, "WINOGRAD_GN", lazy_on)
        seen = []
        orig = ops._lib.call

        def spy(name, *args):
            seen.append(name)
            return orig(name, *args)
        x = x0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
        gam, bet = g0.to(dev).requires_grad_(), b0.to(dev).requires_grad_()
        wt = w0.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
        cb = cb0.to(dev).requires_grad_()
        ops._lib.call = spy
        try:
            hgn = ops.group_norm(x, gam, bet, 32, 1e-6, silu=True, for_conv=co)
            assert isinstance(hgn, ops.DeferredGnOutput) == lazy_on
            y = ops.conv2d(hgn, wt, cb, geom)
            y.backward(dy0.to(dev).contiguous(memory_format=torch.channels_last))
            torch.cuda.synchronize()
        finally:
            ops._lib.call = orig
        out = [t.detach().cpu() for t in (y, x.grad, gam.grad, bet.grad, wt.grad, cb.grad)]
        del x, y, hgn
        torch.cuda.empty_cache()
        return out, seen

    fused, seen = run(True)
    assert "mvae_winograd_input_transform_gn" in seen and "mvae_group_norm_stats_nhwc" in seen
    assert "mvae_group_norm_apply_nhwc" not in seen and "mvae_group_norm_fwd_nhwc" not in seen
    assert "mvae_winograd_input_transform" not in seen  # (the weight gradient read the kept V)
    nch = len(ops._wino_chunks(n, h, w, max(ci, co)))
    assert nch == (2 if ci == 512 else 1) and seen.count("mvae_winograd_input_transform_gn") == nch
    plain, seen2 = run(False)
    assert "mvae_winograd_input_transform_gn" not in seen2
    for a, b in zip(fused, plain):
        assert _rel(a, b.double()) < 5e-5
    y, dx, dgam = fused[0], fused[1], fused[2]
    # float64 GroupNorm + SiLU over the whole batch (in image blocks)
    hs = torch.empty(n, ci, h, w, dtype=torch.float64)
    for b in range(0, n, 32):
        hs[b:b + 32] = F.silu(F.group_norm(x0[b:b + 32].double(), 32, g0.double(), b0.double(), eps=1e-6))
    ws = w0.double()
    ns = torch.randint(0, n, (96,), generator=g)
    oh, ow = torch.randint(0, h, (96,), generator=g), torch.randint(0, w, (96,), generator=g)
    ref = cb0.double()[None, :].repeat(96, 1)
    for r in range(3):
        for s in range(3):
            ref += _gather(hs, ns, _src(oh, r, 1, 1, h, False), _src(ow, s, 1, 1, w, False)) @ ws[:, :, r, s].t()
    assert _rel(y[ns, :, oh, ow], ref) < TOL
    cols = torch.randperm(co, generator=g)[:4]
    ref = torch.zeros(4, ci, 3, 3, dtype=torch.float64)
    for b in range(0, n, 32):
        xp = F.pad(hs[b:b + 32], (1, 1, 1, 1))
        d = dy0[b:b + 32][:, cols].double()
        for r in range(3):
            for s in range(3):
                ref[:, :, r, s] += torch.einsum("nohw,nchw->oc", d, xp[:, :, r:r + h, s:s + w])
    assert _rel(fused[4][cols], ref) < TOL
    del hs
    for i in torch.randperm(n, generator=g)[:2].tolist():
        xr = x0[i:i + 1].double().requires_grad_()
        yr = F.conv2d(F.silu(F.group_norm(xr, 32, g0.double(), b0.double(), eps=1e-6)), ws, cb0.double(), padding=1)
        yr.backward(dy0[i:i + 1].double())
        assert _rel(dx[i:i + 1], xr.grad) < TOL
