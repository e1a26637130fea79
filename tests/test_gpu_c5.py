"""BASELINE config 5 on the HIP path: the c4 architecture (ConditionalVAE 64x64x3, hidden 256, ch_mult 1-2-4-8, 927 M
parameters) trained with precision="bf16-mixed" and the LPIPSWithDiscriminator generator objective over an LPIPS-VGG
network (src/losses/vae_losses.py:67-94 LPIPSLoss, :274-339 generator loss; configs/experiment/multi_modal_cvae.yaml:
24-29; the BASELINE names the VGG backbone). LPIPS weights are synthetic (the pretrained lpips/torchvision weights are
not available offline: LPIPS parity against the package is unpinned).

Tolerances (stated, derived from bf16 operand rounding):
  * single bf16 convolution (fwd / dgrad / wgrad) vs float64 on the SAME bf16-rounded operands: only fp32
    accumulation differs -> 2e-5 relative (sqrt(K) * 2^-24 for K <= 18,432 is ~8e-6);
  * whole c4 forward vs the reference's fp32 golden outputs: every convolution rounds both operands to bf16
    (relative 2^-9 each, so ~2^-8 per layer output) and GroupNorm renormalises between layers, so the per-layer errors
    add like a random walk over the L convolutions on the deepest path: tol = 2^-8 * sqrt(L), L counted from the
    model (~0.03 for c4);
  * LPIPS-VGG distance vs the float64 oracle on the same inputs: 13 bf16 convolutions -> 2^-8 * sqrt(13) ~ 0.014,
    held at 0.03 (the distance is a difference of unit-normalised features)."""
import math

import pytest
import torch
import torch.nn.functional as F

from cases import CASES
from golden_io import golden_state, load_case, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def rel(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def bf(t):
    return t.bfloat16().double()


BF16_CONV_TOL = 2e-5
# n, cin, cout, h, w, k, pad, upsample -- the c5 hot layers (c4 architecture at its three deepest levels) and the
# LPIPS-VGG feature stack at 64x64 input (taps at 64, 32, 16, 8, 4)
C5_LAYERS = [
    (4, 2048, 2048, 8, 8, 3, 1, False),     # encoder/decoder 8x8 level, 2048 channels
    (4, 1024, 1024, 16, 16, 3, 1, False),   # 16x16 level, 1024 channels
    (2, 256, 256, 64, 64, 3, 1, False),     # 64x64 level, 256 channels
    (2, 512, 256, 32, 32, 3, 1, True),      # decoder Upsample 32 -> 64 (sub-pixel form)
    (2, 3, 64, 64, 64, 3, 1, False),        # VGG conv1_1
    (2, 64, 64, 64, 64, 3, 1, False),       # VGG conv1_2
    (2, 128, 128, 32, 32, 3, 1, False),     # VGG conv2_2
    (2, 256, 256, 16, 16, 3, 1, False),     # VGG conv3_x
    (2, 512, 512, 8, 8, 3, 1, False),       # VGG conv4_x
    (2, 512, 512, 4, 4, 3, 1, False),       # VGG conv5_x
]


@pytest.mark.parametrize("case", C5_LAYERS)
def test_bf16_conv_fwd_dgrad_wgrad_at_c5_shapes(dev, case):
    from medvae_disentangled_multimodal_amd import ops
    n, ci, co, h, w, k, p, ups = case
    g = torch.Generator().manual_seed(ci * 7 + co + h)
    x = torch.randn(n, ci, h, w, generator=g)
    wt = torch.randn(co, ci, k, k, generator=g) / math.sqrt(ci * k * k)
    b = torch.randn(co, generator=g) * 0.1
    geom = ops.ConvGeom(k, k, 1, p, p, p, p, ups)
    xd = x.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    wd = wt.to(dev).contiguous(memory_format=torch.channels_last).requires_grad_()
    bd = b.to(dev).requires_grad_()
    prev = ops.set_precision("bf16-mixed")
    try:
        y = ops.conv2d(xd, wd, bd, geom)
        dy = torch.randn(y.shape, generator=g)
        y.backward(dy.to(dev).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(prev)
    assert ops._lib.query("mvae_get_math_mode") == 0
    # float64 reference on the bf16-rounded operands of each GEMM (fwd: x, w; dgrad: dy, w; wgrad: dy, x). The
    # Upsample conv runs in sub-pixel form: its fwd / dgrad GEMM operands are the fp32 tap sums of each parity class
    # (2x2 kernels), rounded to bf16 -- the reference does the same
    xr = bf(x).requires_grad_()
    if ups:
        yr = _subpixel_conv(xr, wt, p) + b.double().view(1, -1, 1, 1)
    else:
        yr = F.conv2d(xr, bf(wt), b.double(), padding=p)
    assert rel(y, yr) < BF16_CONV_TOL
    yr.backward(bf(dy))
    assert rel(xd.grad, xr.grad) < BF16_CONV_TOL
    xg = bf(x)
    wg = bf(wt).requires_grad_()  # wgrad: per-class products of bf16(dy) and bf16(x), taps combined in fp32
    xin = F.interpolate(xg, scale_factor=2.0, mode="nearest") if ups else xg
    F.conv2d(xin, wg, None, padding=p).backward(bf(dy))
    assert rel(wd.grad, wg.grad) < BF16_CONV_TOL
    assert rel(bd.grad, dy.double().sum((0, 2, 3))) < 1e-5


def _subpixel_conv(x, w, pad):
    """nearest-x2 upsample + 3x3 conv (pad 1) as 4 parity classes of 2x2 convs on the low-resolution input, with the
    class kernels summed in fp32 and rounded to bf16 (the bf16 GEMM's operands). x: float64 (already bf16-valued)."""
    assert pad == 1
    n, _, h, wd = x.shape
    co = w.shape[0]
    # rows feeding output parity 0: source i-1 <- tap 0, source i <- taps 1 + 2; parity 1: i <- 0 + 1, i+1 <- 2
    groups = {0: ((0,), (1, 2)), 1: ((0, 1), (2,))}
    y = x.new_zeros(n, co, 2 * h, 2 * wd)
    for ph in (0, 1):
        for pw in (0, 1):
            k = torch.zeros(co, w.shape[1], 2, 2)
            for a, rs in enumerate(groups[ph]):
                for c, ss in enumerate(groups[pw]):
                    k[:, :, a, c] = sum(w[:, :, r, s] for r in rs for s in ss)
            xp = F.pad(x, (1 - pw, pw, 1 - ph, ph))
            y[:, :, ph::2, pw::2] = F.conv2d(xp, k.bfloat16().double())
    return y


def _conv_depth(model) -> int:
    """Convolutions on the deepest encoder -> decoder path (ResnetBlock: 2, AttnBlock: q/k/v + proj_out = 2 in
    sequence, Down/Upsample: 1, conv_in / conv_out: 1 each side)."""
    n = 0
    for name, m in model.named_modules():
        if name.endswith(("conv1", "conv2", "conv_in", "conv_out")) or name.endswith(("downsample.conv", "upsample.conv")):
            n += 1
        elif name.endswith(("proj_out", ".q")):
            n += 1
    return n


def _c5_module(dev, meta, case):
    import medvae_disentangled_multimodal_amd as M
    model = getattr(M, case["cls"])(**case["kwargs"])
    model.load_state_dict(golden_state(meta))
    model = model.to(dev)
    loss = dict(type="lpips_discriminator", perceptual_factor=1.0, kl_factor=1e-5, discriminator_iter_start=10000,
                allow_synthetic_lpips=True, lpips_net="vgg")
    mod = M.VAELightningModule(model, dict(type="adamw", lr=1e-4, weight_decay=1e-5, betas=[0.5, 0.999]),
                               {"type": "none"}, loss, gradient_clip_val=1.0, precision="bf16-mixed")
    mod.configure_optimizers()
    return mod


def test_c5_bf16_lpips_vgg_step_on_c4_architecture(dev):
    """cvae_c4_full weights / batch / eps (B=2, the exact BASELINE c4 architecture) in bf16-mixed with the LPIPS-VGG
    generator objective: forward outputs vs the reference's fp32 golden outputs at the bf16 tolerance, the objective's
    terms vs float64 restatements on the same tensors, then two finite fit_steps with the math mode restored."""
    from medvae_disentangled_multimodal_amd import ops
    from oracle.torch_ref import lpips_vgg
    meta, data = load_case("cvae_c4_full")
    case = CASES["cvae_c4_full"]
    mod = _c5_module(dev, meta, case)
    x = torch.from_numpy(data["in.x"]).to(dev)
    oh = torch.from_numpy(data["in.cond"]).to(dev)
    batch = (x, torch.zeros(x.shape[0], 1, dtype=torch.long, device=dev), oh)
    eps = torch.from_numpy(data["in.eps"]).to(dev)
    depth = _conv_depth(mod.model)
    tol = 2.0 ** -8 * math.sqrt(depth)
    assert 40 <= depth <= 120 and tol < 0.05

    prev = ops.set_precision("bf16-mixed")
    try:
        loss = mod.training_step(batch, 0, eps=eps)
        torch.cuda.synchronize()
    finally:
        ops.restore_math_mode(prev)
    out = mod._last_outputs
    errs = {k: rel_err(out[k].detach().cpu(), data[f"out.{k}"]) for k in ("reconstruction", "mean", "logvar", "z")}
    assert all(v < tol for v in errs.values()), (errs, tol)
    assert any(v > 1e-5 for v in errs.values()), "bf16 arithmetic should be visible against the fp32 reference"
    # objective terms on the HIP path's own tensors: KL closed form (float64) and LPIPS-VGG (float64 oracle)
    mu, lv = out["mean"].detach().double().cpu(), out["logvar"].detach().double().cpu()
    kl_ref = float(-0.5 * (1 + lv - mu ** 2 - lv.exp()).sum() / x.shape[0])
    kl = float(mod.logged["train/kl_loss"])
    assert abs(kl - kl_ref) <= 1e-5 * abs(kl_ref)
    lp = mod.criterion.perceptual_loss.lpips
    W = {k: v.detach().double().cpu() for k, v in lp.internal_weights().items()}
    p_ref = float(lpips_vgg(W, x.double().cpu(), out["reconstruction"].detach().double().cpu()).mean())
    p = float(mod.logged["train/p_loss"])
    assert abs(p - p_ref) <= 0.03 * abs(p_ref), (p, p_ref)
    assert abs(float(loss) - (p + 1e-5 * kl)) <= 1e-5 * abs(float(loss))

    l0 = float(mod.fit_step(batch, 0, eps=eps))
    l1 = float(mod.fit_step(batch, 1, eps=eps))
    assert math.isfinite(l0) and math.isfinite(l1)
    assert mod.optimizer.last_total_norm is not None and math.isfinite(float(mod.optimizer.last_total_norm))
    assert ops._lib.query("mvae_get_math_mode") == 0
    assert mod.global_step_count == 2
