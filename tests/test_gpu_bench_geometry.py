"""Hot-path numerics at the bench's own geometry (c4: batch 256, 64x64 input). The GEMM planner picks tiles and
split-K factors from M = B*H*W, so the launches the bench times (M = 16,384 at the 8x8x2048 level, 65,536 at 16x16,
1,048,576 for the 32 -> 64 Upsample) differ from the small-batch parity cases. Here the three hottest c4 convolutions
run at B=256 in the default fp32-class (3xBF16) arithmetic -- forward, input gradient and weight gradient through
the same ops.conv2d autograd path the model uses -- and are checked against float64 on a sampled subset: output rows
(pixels x all channels), input-gradient rows, and weight-gradient columns (output channels x all taps / inputs).
Tolerance 2e-4 relative per sampled block (the CONV_TOL of tests/test_gpu_kernels.py).
The two deepest layers also run in the bf16-mixed arithmetic (config 5; forward and input gradient on packed bf16
operands through the LDS-DMA GEMM main loop): the float64 reference then uses the bf16-rounded operands of each
GEMM, so only fp32 accumulation differs -- tolerance 1e-4 (sqrt(K) * 2^-24 for K = 18,432 is ~8e-6)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
TOL = 2e-4

# n, cin, cout, h, w (input), upsample -- encoder/decoder 8x8x2048, 16x16x1024, decoder Upsample 32 -> 64 at 512 ch
LAYERS = [(256, 2048, 2048, 8, 8, False), (256, 1024, 1024, 16, 16, False), (256, 512, 512, 32, 32, True)]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _src(o, r, pad, size, ups):
    """input index feeding output o through tap r (stride 1, pad, optional nearest x2 upsample), or -1."""
    u = o - pad + r
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


@pytest.mark.parametrize("layer,prec", [(l, "32") for l in LAYERS] + [(l, "bf16-mixed") for l in LAYERS[:2]])
def test_c4_hot_conv_at_batch_256(dev, layer, prec):
    from medvae_disentangled_multimodal_amd import ops
    n, ci, co, h, w, ups = layer
    tol = TOL if prec == "32" else 1e-4
    g = torch.Generator().manual_seed(ci + h)
    x = torch.randn(n, ci, h, w, generator=g)
    wt = torch.randn(co, ci, 3, 3, generator=g) / math.sqrt(ci * 9)
    b = torch.randn(co, generator=g) * 0.1
    ho, wo = (2 * h, 2 * w) if ups else (h, w)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, ups)
    xd = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    wd = wt.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    bd = b.to(dev).requires_grad_()
    dy = torch.randn(n, co, ho, wo, generator=g)
    prev = ops.set_precision(prec)
    try:
        y = ops.conv2d(xd, wd, bd, geom)
        y.backward(dy.to(dev).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(prev)
    assert ops._lib.query("mvae_get_math_mode") == 0

    if prec == "32":
        xs, ws, dys = x.double(), wt.double(), dy.double()
    else:
        xs, ws, dys = x.bfloat16().double(), wt.bfloat16().double(), dy.bfloat16().double()
    ns = torch.randint(0, n, (96,), generator=g)
    # forward rows: y[n, :, oh, ow] = sum_{r,s} W[:, :, r, s] x_src(n, oh, ow, r, s) + b
    oh, ow = torch.randint(0, ho, (96,), generator=g), torch.randint(0, wo, (96,), generator=g)
    ref = b.double()[None, :].repeat(96, 1)
    for r in range(3):
        for s in range(3):
            ref += _gather(xs, ns, _src(oh, r, 1, h, ups), _src(ow, s, 1, w, ups)) @ ws[:, :, r, s].t()
    got = y.detach()[ns.to(dev), :, oh.to(dev), ow.to(dev)].cpu()
    assert _rel(got, ref) < tol
    # input-gradient rows: dx[n, :, ih, iw] = sum over (upsampled copy a, b) and taps of dy at the output it fed
    ih, iw = torch.randint(0, h, (96,), generator=g), torch.randint(0, w, (96,), generator=g)
    ref = torch.zeros(96, ci, dtype=torch.float64)
    copies = (0, 1) if ups else (0,)
    for a in copies:
        for c in copies:
            uh, uw = (2 * ih + a, 2 * iw + c) if ups else (ih, iw)
            for r in range(3):
                for s in range(3):
                    o_h, o_w = uh + 1 - r, uw + 1 - s
                    ok = (o_h >= 0) & (o_h < ho) & (o_w >= 0) & (o_w < wo)
                    v = dys[ns, :, o_h.clamp(0, ho - 1), o_w.clamp(0, wo - 1)] * ok[:, None].double()
                    ref += v @ ws[:, :, r, s]
    got = xd.grad[ns.to(dev), :, ih.to(dev), iw.to(dev)].cpu()
    assert _rel(got, ref) < tol
    # weight-gradient columns: dW[o, :, r, s] = sum over all n, oh, ow of dy[n, o, oh, ow] x_src(n, oh, ow, r, s)
    cols = torch.randperm(co, generator=g)[:4]
    ref = torch.zeros(4, ci, 3, 3, dtype=torch.float64)
    xin = F.interpolate(xs, scale_factor=2.0, mode="nearest") if ups else xs
    for n0 in range(0, n, 32):
        xp = F.pad(xin[n0:n0 + 32], (1, 1, 1, 1))
        d = dys[n0:n0 + 32][:, cols]  # [32, 4, ho, wo]
        for r in range(3):
            for s in range(3):
                ref[:, :, r, s] += torch.einsum("nohw,nchw->oc", d, xp[:, :, r:r + ho, s:s + wo])
    got = wd.grad[cols.to(dev)].cpu()
    assert _rel(got, ref) < tol
    assert _rel(bd.grad.cpu(), dy.double().sum((0, 2, 3))) < 1e-5
