"""LPIPS (perceptual loss, config 5) and the bf16 GEMM mode on the MI355X, against the CPU oracle
(oracle/torch_ref.py:lpips_alex, a restatement of lpips 0.1.4; parity vs the real package is
unpinned) and plain torch references.

Tolerances: elementwise / pooling kernels exact; the per-layer distance 1e-5 (fp32 reductions);
the full network 2e-3 relative (five 3xBF16 convolutions deep); bf16 mode against a float64
reference on bf16-rounded operands 1e-5.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def cl(t, dev):
    return t.to(dev).contiguous(memory_format=torch.channels_last)


def rel(a, b):
    a = a.detach().double().cpu().flatten()
    b = b.detach().double().cpu().flatten()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def test_relu_maxpool_exact(dev):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 40, 15, 15, generator=g)
    x[0, 0, :3, :3] = 1.0  # ties inside a window: first max wins, as in torch
    xd = cl(x, dev).requires_grad_()
    y = ops.max_pool3s2(ops.relu(xd))
    xr = x.clone().requires_grad_()
    yr = F.max_pool2d(F.relu(xr), 3, 2)
    assert y.shape == yr.shape
    assert torch.equal(y.cpu(), yr)
    dy = torch.randn(yr.shape, generator=g)
    y.backward(cl(dy, dev))
    yr.backward(dy)
    assert torch.allclose(xd.grad.cpu(), xr.grad, atol=1e-6, rtol=0)


def test_lpips_layer_distance(dev):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(5)
    f0 = torch.relu(torch.randn(3, 192, 7, 7, generator=g))
    f1 = torch.relu(torch.randn(3, 192, 7, 7, generator=g))
    w = torch.rand(192, generator=g) / 192
    a = cl(f0, dev).requires_grad_()
    b = cl(f1, dev).requires_grad_()
    s = ops.lpips_dist(a, b, w.to(dev))
    gs = torch.tensor([0.5, -1.0, 2.0])
    s.backward(gs.to(dev))

    f0r, f1r = f0.double().requires_grad_(), f1.double().requires_grad_()
    n0 = f0r / (f0r.pow(2).sum(1, keepdim=True).sqrt() + 1e-10)
    n1 = f1r / (f1r.pow(2).sum(1, keepdim=True).sqrt() + 1e-10)
    sr = ((n0 - n1) ** 2 * w.double().view(1, -1, 1, 1)).sum(1).mean((1, 2))
    sr.backward(gs.double())
    assert rel(s, sr) < 1e-5
    assert rel(a.grad, f0r.grad) < 1e-5
    assert rel(b.grad, f1r.grad) < 1e-5


def _lpips_weights(m):
    return {k: v.detach().cpu().double() for k, v in m.internal_weights().items()}


def test_lpips_network_vs_oracle(dev):
    from medvae_disentangled_multimodal_amd.losses import LPIPSLoss
    from oracle.torch_ref import lpips_alex
    loss = LPIPSLoss(allow_synthetic=True, seed=7)
    g = torch.Generator().manual_seed(11)
    x = torch.rand(2, 3, 64, 64, generator=g)
    rec = (x + 0.2 * torch.randn(x.shape, generator=g)).clamp(0, 1)
    rd = cl(rec, dev).requires_grad_()
    v = loss(cl(x, dev), rd)
    v.backward()

    W = _lpips_weights(loss.lpips)
    rr = rec.double().requires_grad_()
    vr = lpips_alex(W, x.double(), rr).mean()
    vr.backward()
    assert abs(float(v) - float(vr)) / abs(float(vr)) < 2e-3
    assert rel(rd.grad, rr.grad) < 5e-3
    # identical inputs -> zero distance
    assert float(loss(cl(x, dev), cl(x, dev))) < 1e-6


def test_lpips_vgg_vs_oracle(dev):
    from medvae_disentangled_multimodal_amd.losses import LPIPSLoss
    from oracle.torch_ref import lpips_vgg
    loss = LPIPSLoss(net="vgg", allow_synthetic=True, seed=9)
    g = torch.Generator().manual_seed(12)
    x = torch.rand(2, 3, 64, 64, generator=g)
    rec = (x + 0.2 * torch.randn(x.shape, generator=g)).clamp(0, 1)
    rd = cl(rec, dev).requires_grad_()
    v = loss(cl(x, dev), rd)
    v.backward()
    W = _lpips_weights(loss.lpips)
    rr = rec.double().requires_grad_()
    vr = lpips_vgg(W, x.double(), rr).mean()
    vr.backward()
    assert abs(float(v) - float(vr)) / abs(float(vr)) < 2e-3
    assert rel(rd.grad, rr.grad) < 5e-3


def test_maxpool_2x2(dev):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 24, 9, 8, generator=g)
    xd = cl(x, dev).requires_grad_()
    y = ops.max_pool(xd, 2, 2)
    xr = x.clone().requires_grad_()
    yr = F.max_pool2d(xr, 2, 2)
    assert torch.equal(y.cpu(), yr)
    dy = torch.randn(yr.shape, generator=g)
    y.backward(cl(dy, dev))
    yr.backward(dy)
    assert torch.equal(xd.grad.cpu(), xr.grad)


def test_lpips_gray_input_repeats_channels(dev):
    from medvae_disentangled_multimodal_amd.losses import LPIPSLoss
    loss = LPIPSLoss(allow_synthetic=True, seed=1)
    g = torch.Generator().manual_seed(2)
    x = torch.rand(2, 1, 32, 32, generator=g)
    y = torch.rand(2, 1, 32, 32, generator=g)
    a = loss(cl(x, dev), cl(y, dev))
    b = loss(cl(x.repeat(1, 3, 1, 1), dev), cl(y.repeat(1, 3, 1, 1), dev))
    assert float(a) == pytest.approx(float(b), rel=1e-6)


def test_lpips_refuses_without_weights():
    from medvae_disentangled_multimodal_amd.lpips import LPIPS
    import os
    if os.environ.get("MVAE_LPIPS_WEIGHTS"):
        pytest.skip("weights configured")
    with pytest.raises(RuntimeError):
        LPIPS()


def test_bf16_math_mode_conv(dev):
    """precision='bf16-mixed': the conv GEMM takes bf16-rounded operands, fp32 accumulation."""
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(13)
    x = torch.randn(4, 64, 16, 16, generator=g)
    w = torch.randn(96, 64, 3, 3, generator=g) / 24
    b = torch.randn(96, generator=g)
    geom = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1)
    prev = ops.set_precision("bf16-mixed")
    try:
        y = ops.conv2d(cl(x, dev), cl(w, dev), b.to(dev), geom)
    finally:
        ops.restore_math_mode(prev)
    ref = F.conv2d(x.bfloat16().double(), w.bfloat16().double(), b.double(), padding=1)
    assert rel(y, ref) < 1e-5
    # and it really is bf16 arithmetic: the fp32 result differs at the bf16 rounding level
    y32 = ops.conv2d(cl(x, dev), cl(w, dev), b.to(dev), geom)
    r32 = F.conv2d(x.double(), w.double(), b.double(), padding=1)
    assert rel(y32, r32) < 2e-4 < rel(y, r32)
    assert ops._lib.query("mvae_get_math_mode") == 0


def test_lpips_generator_step(dev):
    """Config-5 objective (LPIPS + KL.sum()/B generator loss, bf16 GEMMs) through fit_step."""
    import medvae_disentangled_multimodal_amd as M
    torch.manual_seed(0)
    model = M.ConditionalVAE(input_channels=3, latent_dim=8, hidden_channels=32, ch_mult=(1, 2), num_res_blocks=1,
                             attn_resolutions=[], resolution=32, condition_dim=12).to(dev)
    mod = M.VAELightningModule(model, {"type": "adamw", "lr": 1e-4}, {"type": "none"},
                               {"type": "lpips_discriminator", "perceptual_factor": 1.0, "kl_factor": 1e-5,
                                "discriminator_iter_start": 10000, "allow_synthetic_lpips": True},
                               gradient_clip_val=1.0, precision="bf16-mixed")
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.rand(4, 3, 32, 32, device=dev, generator=g) * 2 - 1
    idx = torch.randint(0, 5, (4,), device=dev, generator=g)
    onehot = F.one_hot(idx, 12).float()
    l0 = float(mod.fit_step((x, idx.view(-1, 1), onehot), 0))
    l1 = float(mod.fit_step((x, idx.view(-1, 1), onehot), 1))
    assert torch.isfinite(torch.tensor([l0, l1])).all()
    assert "train/p_loss" in mod.logged and "train/kl_loss" in mod.logged
    assert M.ops._lib.query("mvae_get_math_mode") == 0
