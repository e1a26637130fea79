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
(sqrt(K) * 2^-24 for K = 18,432 is ~8e-6)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
TOL = 2e-4

# n, cin, cout, h, w (input), k, stride, pads (t, l, b, r), upsample
C4 = [(256, 2048, 2048, 8, 8, 3, 1, (1, 1, 1, 1), False), (256, 1024, 1024, 16, 16, 3, 1, (1, 1, 1, 1), False),
      (256, 512, 512, 32, 32, 3, 1, (1, 1, 1, 1), True)]
C2 = [(256, 512, 512, 7, 7, 3, 1, (1, 1, 1, 1), False), (256, 512, 512, 7, 7, 1, 1, (0, 0, 0, 0), False),
      (256, 128, 128, 28, 28, 3, 1, (1, 1, 1, 1), False), (256, 128, 128, 28, 28, 3, 2, (0, 0, 1, 1), False),
      (256, 256, 256, 14, 14, 3, 1, (1, 1, 1, 1), True), (256, 512, 256, 7, 7, 3, 1, (1, 1, 1, 1), False)]
C3 = [(512, 32, 32, 28, 28, 3, 1, (1, 1, 1, 1), False), (512, 64, 64, 14, 14, 3, 1, (1, 1, 1, 1), False),
      (512, 128, 128, 7, 7, 3, 1, (1, 1, 1, 1), False), (512, 128, 128, 7, 7, 1, 1, (0, 0, 0, 0), False),
      (512, 32, 32, 28, 28, 3, 2, (0, 0, 1, 1), False), (512, 64, 64, 14, 14, 3, 1, (1, 1, 1, 1), True)]
# bf16-mixed (config 5): the c4 layers above plus a 64 x 32x32 x 256 layer (fwd M = 65,536: 256 tiles of 256x256) and
# its stride-2 Downsample, every pass on the LDS-DMA main loop
C5 = C4[:2] + [(64, 256, 256, 32, 32, 3, 1, (1, 1, 1, 1), False), (64, 256, 256, 64, 64, 3, 2, (0, 0, 1, 1), False)]
LAYERS = [("c4", l, "32") for l in C4] + [("c5", l, "bf16-mixed") for l in C5] + \
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
    prev = ops.set_precision(prec)
    try:
        y = ops.conv2d(xd, wd, bd, geom)
        y.backward(dy.to(dev).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(prev)
    assert ops._lib.query("mvae_get_math_mode") == 0
    assert tuple(y.shape) == (n, co, ho, wo)

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
