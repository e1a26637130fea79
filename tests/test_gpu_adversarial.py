"""Adversarial branch (row (f)2) on the MI355X vs the oracle (oracle/torch_ref.py: discriminator,
hinge_d_loss -- restating src/models/discriminator.py and vae_losses.py:297-382) with the same
weights: BatchNorm(+LeakyReLU) forward/backward, running statistics, the PatchGAN forward/backward,
the hinge loss and its gradient, and a full manual generator + discriminator step."""
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


def test_batch_norm_leaky(dev):
    from medvae_disentangled_multimodal_amd import ops
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 96, 6, 5, generator=g) * 2 + 0.5
    gam, bet = torch.rand(96, generator=g) + 0.5, torch.randn(96, generator=g)
    rm, rv = torch.zeros(96), torch.ones(96)
    xd = cl(x, dev).requires_grad_()
    gd, bd = gam.to(dev).requires_grad_(), bet.to(dev).requires_grad_()
    rmd, rvd = rm.to(dev), rv.to(dev)
    y = ops.batch_norm(xd, gd, bd, rmd, rvd, True, 0.1, 1e-5, 0.2)
    xr, gr, br = x.double().requires_grad_(), gam.double().requires_grad_(), bet.double().requires_grad_()
    rmr, rvr = rm.double(), rv.double()
    yr = F.leaky_relu(F.batch_norm(xr, rmr, rvr, gr, br, True, 0.1, 1e-5), 0.2)
    assert rel(y, yr) < 1e-5
    assert rel(rmd, rmr) < 1e-5 and rel(rvd, rvr) < 1e-5
    dy = torch.randn(x.shape, generator=g)
    y.backward(cl(dy, dev))
    yr.backward(dy.double())
    assert rel(xd.grad, xr.grad) < 1e-4
    assert rel(gd.grad, gr.grad) < 1e-4 and rel(bd.grad, br.grad) < 1e-4
    # eval mode: running statistics
    ye = ops.batch_norm(cl(x, dev), gd.detach(), bd.detach(), rmd, rvd, False, 0.1, 1e-5, -1.0)
    yre = F.batch_norm(x.double(), rmr, rvr, gam.double(), bet.double(), False, 0.1, 1e-5)
    assert rel(ye, yre) < 1e-5


def test_discriminator_vs_oracle(dev):
    from medvae_disentangled_multimodal_amd.discriminator import NLayerDiscriminator
    from oracle import torch_ref as R
    torch.manual_seed(3)
    D = NLayerDiscriminator().to(dev)
    names = [k for k, _ in D.state_dict().items()]
    assert names[:4] == ["main.0.weight", "main.0.bias", "main.2.weight", "main.2.bias"]
    assert "main.3.running_mean" in names and "main.11.weight" in names
    W = {k: v.detach().cpu().double().clone() for k, v in D.state_dict().items()}
    g = torch.Generator().manual_seed(4)
    x = torch.rand(2, 3, 64, 64, generator=g) * 2 - 1
    xd = cl(x, dev).requires_grad_()
    out = D(xd)
    xr = x.double().requires_grad_()
    Wr = {k: v.requires_grad_() if v.is_floating_point() and "running" not in k else v for k, v in W.items()}
    running = {k: v for k, v in W.items() if "running" in k}
    outr = R.discriminator(Wr, xr, running=running)
    assert out.shape == outr.shape == (2, 1, 6, 6)
    assert rel(out, outr) < 1e-3
    assert rel(D.main[3].running_var, running["main.3.running_var"]) < 1e-5
    loss = F.mse_loss(out, torch.zeros_like(out))
    loss.backward()
    F.mse_loss(outr, torch.zeros_like(outr)).backward()
    assert rel(xd.grad, xr.grad) < 2e-3
    assert rel(D.main[5].weight.grad, Wr["main.5.weight"].grad) < 2e-3


def test_hinge_and_generator_terms(dev):
    from medvae_disentangled_multimodal_amd import ops
    from oracle import torch_ref as R
    g = torch.Generator().manual_seed(8)
    a = (torch.randn(3, 1, 6, 6, generator=g) * 2).to(dev).requires_grad_()
    b = (torch.randn(3, 1, 6, 6, generator=g) * 2).to(dev).requires_grad_()
    d = 0.5 * (ops.hinge_real(a) + ops.hinge_fake(b))
    ar, br = a.detach().cpu().double().requires_grad_(), b.detach().cpu().double().requires_grad_()
    dr = R.hinge_d_loss(ar, br)
    assert float(d) == pytest.approx(float(dr), rel=1e-6)
    d.backward()
    dr.backward()
    assert rel(a.grad, ar.grad) < 1e-6 and rel(b.grad, br.grad) < 1e-6
    gl = ops.neg_mean(a)
    assert float(gl) == pytest.approx(-float(a.mean()), rel=1e-6)


def test_adversarial_fit_step(dev):
    import medvae_disentangled_multimodal_amd as M
    torch.manual_seed(0)
    model = M.ConditionalVAE(input_channels=3, latent_dim=8, hidden_channels=32, ch_mult=(1, 2), num_res_blocks=1,
                             attn_resolutions=[], resolution=32).to(dev)
    mod = M.VAELightningModule(model, {"type": "adam", "lr": 1e-4}, {"type": "none"},
                               {"type": "lpips_discriminator", "perceptual_factor": 1.0, "kl_factor": 1e-5,
                                "discriminator_iter_start": 0, "allow_synthetic_lpips": True,
                                "discriminator": {"input_nc": 3, "ndf": 16, "n_layers": 2}})
    mod.configure_optimizers()
    d0 = mod.flat_d.data.clone()
    v0 = mod.flat.data.clone()
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.rand(4, 3, 32, 32, device=dev, generator=g) * 2 - 1
    idx = torch.randint(0, 5, (4,), device=dev, generator=g)
    batch = (x, idx.view(-1, 1), F.one_hot(idx, 12).float())
    loss = mod.fit_step(batch, 0)
    assert torch.isfinite(loss)
    for k in ("train/g_loss", "train/d_weight", "train/d_loss", "train/p_loss"):
        assert k in mod.logged and torch.isfinite(torch.as_tensor(mod.logged[k])), k
    assert float(mod.logged["train/d_weight"]) > 0
    assert not torch.equal(mod.flat_d.data, d0) and not torch.equal(mod.flat.data, v0)
    assert mod.global_step_count == 2
    mod.fit_step(batch, 1)
    assert mod.global_step_count == 4
