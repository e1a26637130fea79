"""Fused glue of the disentangled training step against the torch compositions it replaces.

* ops.latent_prep (csrc/loss.hip latent_prep_fwd / _bwd): encode's NaN scrub, forward's clamps of mu / logvar, the
  reparameterization and the posterior's clamped std (src/models/disentangled_conditional_vae.py:255-301, 388-398;
  base_vae.py:83-87) in one launch per direction; checked with NaN / +-inf / out-of-range encoder outputs, every
  combination of incoming gradients, and a strided (channel-slice) encoder output.
* ops.loss_combine (loss_combine_fwd / _bwd): DisentangledVAELoss's finite-or-zero terms, weighted total and total
  guard (:528-570), with NaN / inf terms and an overflowing total.

Tolerance: the same fp32 arithmetic as torch's elementwise kernels up to 1 ulp (expf vs torch.exp, and the kernel's
fused multiply-add in z = mu + eps * s where torch rounds the product first): rtol 1e-6 / atol 1e-6 on values of
magnitude <= 10 (1 ulp at 10 is 9.5e-7); selections (masks, replaced values) exact.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

RTOL, ATOL = 1e-6, 1e-6


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _torch_latent(h, eps, zc):
    mu, lv = torch.chunk(h, 2, dim=1)
    mu = torch.where(torch.isnan(mu), 0.0, mu)
    lv = torch.where(torch.isnan(lv), 0.0, lv)
    lv = torch.clamp(lv, min=-10.0, max=10.0)
    mu = torch.clamp(mu, min=-10.0, max=10.0)
    z = mu + eps * torch.exp(0.5 * lv)
    std = torch.clamp(torch.exp(0.5 * lv), min=1e-6, max=10.0)
    return mu, lv, std, z


def _encoder_out(dev, n=6, zc=16, r=7, wide=0, seed=0):
    g = torch.Generator().manual_seed(seed)
    h = torch.randn(n, 2 * zc + wide, r, r, generator=g) * 6.0  # a good share beyond +-10 after the scale below
    h[:, :, 0, 0] *= 3.0
    flat = h.view(-1)
    idx = torch.randperm(flat.numel(), generator=g)
    flat[idx[:20]] = float("nan")
    flat[idx[20:30]] = float("inf")
    flat[idx[30:40]] = -float("inf")
    flat[idx[40:50]] = 10.0
    flat[idx[50:60]] = -10.0
    # logvar entries whose std hits the [1e-6, 10] clamp: exp(0.5 lv) > 10 <=> lv > 4.6
    h = h.to(dev).contiguous(memory_format=torch.channels_last)
    if wide:
        h = h[:, :2 * zc]  # channel slice of a wider NHWC output: row stride 2 zc + wide
    eps = torch.randn(n, zc, r, r, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    return h, eps


@pytest.mark.parametrize("wide", [0, 4])
@pytest.mark.parametrize("grads", ["all", "mu_lv_z", "z_only", "std_only"])
def test_latent_prep_matches_torch(wide, grads):
    from medvae_disentangled_multimodal_amd import ops
    dev = _dev()
    zc = 16
    h0, eps = _encoder_out(dev, zc=zc, wide=wide)
    h_t = h0.detach().clone().requires_grad_()
    h_f = h0.detach().clone().requires_grad_()
    ref = _torch_latent(h_t, eps, zc)
    got = ops.latent_prep(h_f, zc, eps)
    for a, b in zip(got, ref):
        assert a.shape == b.shape
        torch.testing.assert_close(a, b, rtol=RTOL, atol=ATOL, equal_nan=False)
    g = torch.Generator().manual_seed(3)
    gs = [torch.randn(ref[0].shape, generator=g).to(dev) for _ in range(4)]
    use = {"all": (1, 1, 1, 1), "mu_lv_z": (1, 1, 0, 1), "z_only": (0, 0, 0, 1), "std_only": (0, 0, 1, 0)}[grads]
    out_r = sum(((o * gg).sum() for o, gg, u in zip(ref, gs, use) if u), torch.zeros((), device=dev))
    out_f = sum(((o * gg).sum() for o, gg, u in zip(got, gs, use) if u), torch.zeros((), device=dev))
    (dr,) = torch.autograd.grad(out_r, h_t)
    (df,) = torch.autograd.grad(out_f, h_f)
    assert torch.isfinite(df).all()
    torch.testing.assert_close(df, dr, rtol=1e-5, atol=1e-6)
    # the masked entries (NaN, +-inf, beyond +-10) get exactly zero
    bad = ~torch.isfinite(h0) | (h0.abs() > 10)
    assert (df[bad] == 0).all()


def test_latent_prep_in_the_model_matches_the_torch_chain(monkeypatch):
    """DisentangledConditionalVAE.forward with the fused latent side = the torch chain (MVAE_NO_LATENT_PREP path)."""
    from medvae_disentangled_multimodal_amd import disentangled as dm
    dev = _dev()
    torch.manual_seed(0)
    model = dm.DisentangledConditionalVAE(num_modalities=5, shared_latent_dim=8, modality_latent_dim=8,
                                          hidden_channels=32, ch_mult=(1, 2, 4), num_res_blocks=1,
                                          attn_resolutions=[], dropout=0.0, resolution=28).to(dev)
    g = torch.Generator().manual_seed(1)
    x = (torch.rand(8, 3, 28, 28, generator=g) * 2 - 1).to(dev)
    idx = torch.tensor([0, 1, 2, 3, 4, 1, 0, 2], device=dev)
    eps = torch.randn(8, 16, 7, 7, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    outs = {}
    for fused in (True, False):
        monkeypatch.setattr(dm, "LATENT_PREP", fused)
        model.zero_grad(set_to_none=True)
        o = model(x, idx, eps=eps)
        loss = (o["reconstruction"] ** 2).mean() + (o["mu"] ** 2).mean() + o["logvar"].exp().mean() + \
            o["posterior"].stddev.mean()
        loss.backward()
        outs[fused] = (o["z"].detach().clone(), o["posterior"].stddev.detach().clone(),
                       model.encoder.conv_out.weight.grad.detach().clone())
    for a, b in zip(outs[True], outs[False]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def _torch_combine(terms, w):
    fz = [torch.where(torch.isfinite(t), t, 0.0) for t in terms]
    tot = w[0] * fz[0] + w[1] * fz[1] + w[2] * fz[2] + w[3] * fz[3]
    tot = torch.where(torch.isfinite(tot), tot, 1e6)
    return [tot] + fz


@pytest.mark.parametrize("case", ["finite", "nan_sep", "inf_recon", "overflow_total", "all_bad"])
def test_loss_combine_matches_torch(case):
    from medvae_disentangled_multimodal_amd import ops
    dev = _dev()
    vals = {"finite": [0.31, 0.012, -1.7, 2.3], "nan_sep": [0.31, 0.012, math.nan, 2.3],
            "inf_recon": [math.inf, 0.012, -1.7, 2.3], "overflow_total": [3e38, 0.5, -1.7, 3e38],
            "all_bad": [math.nan, math.inf, -math.inf, math.nan]}[case]
    w = [1.0, 1.0, 0.1, 0.05] if case != "overflow_total" else [1.0, 1.0, 0.1, 1.0]
    base = [torch.tensor(v, device=dev) for v in vals]
    tr = [b.clone().requires_grad_() for b in base]
    tf = [b.clone().requires_grad_() for b in base]
    ref = _torch_combine(tr, w)
    got = ops.loss_combine(tf, w)
    for a, b in zip(got, ref):
        assert a.shape == b.shape == ()
        torch.testing.assert_close(a, b, rtol=0, atol=0)  # same fp32 operations in the same order
    gg = [1.0, 0.25, -0.5, 2.0, 0.0]  # d/d(total), d/d(logged terms)
    sr = sum(o * c for o, c in zip(ref, gg))
    sf = sum(o * c for o, c in zip(got, gg))
    gr = torch.autograd.grad(sr, tr)
    gf = torch.autograd.grad(sf, tf)
    for a, b in zip(gf, gr):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


def test_loss_combine_total_only_backward():
    from medvae_disentangled_multimodal_amd import ops
    dev = _dev()
    ts = [torch.tensor(v, device=dev, requires_grad=True) for v in (0.5, 0.25, 0.125, 1.0)]
    tot = ops.loss_combine(ts, [1.0, 6.0, 0.1, 0.05])[0]
    tot.backward()
    assert [float(t.grad) for t in ts] == pytest.approx([1.0, 6.0, 0.1, 0.05], rel=1e-7)


def test_loss_combine_second_backward_through_retained_graph():
    """autograd.grad with retain_graph, then backward through the same graph (the torch composition allows it)."""
    from medvae_disentangled_multimodal_amd import ops
    dev = _dev()
    ts = [torch.tensor(v, device=dev, requires_grad=True) for v in (0.5, float("nan"), 0.125)]
    tot = ops.loss_combine(ts, [1.0, 6.0, 0.1])[0]
    g1 = torch.autograd.grad(tot, ts, retain_graph=True)
    tot.backward()
    assert [float(g) for g in g1] == pytest.approx([1.0, 0.0, 0.1], rel=1e-7)
    assert [float(t.grad) for t in ts] == pytest.approx([1.0, 0.0, 0.1], rel=1e-7)


# ---- batched dgrad weight re-layouts (ops._TransposedWeights, mvae_conv_weight_transpose_batched) -------------------
_CVAE = dict(input_channels=3, latent_dim=8, hidden_channels=32, ch_mult=(1, 2, 4), num_res_blocks=1,
             attn_resolutions=[14], dropout=0.0, resolution=28, condition_method="concat")
_DIS = dict(num_modalities=5, shared_latent_dim=8, modality_latent_dim=8, hidden_channels=32, ch_mult=(1, 2, 4),
            num_res_blocks=1, attn_resolutions=[], dropout=0.0, resolution=28, modality_separation_weight=0.1,
            contrastive_weight=0.05)


@pytest.mark.parametrize("cls,kw,loss,prec", [
    ("ConditionalVAE", _CVAE, dict(type="vae", recon_loss_type="mse", kl_weight=1.0, recon_weight=1.0), "32"),
    ("ConditionalVAE", _CVAE, dict(type="vae", recon_loss_type="mse", kl_weight=1.0, recon_weight=1.0), "bf16-mixed"),
    ("DisentangledConditionalVAE", _DIS, dict(type="disentangled_vae", recon_loss_type="mse", kl_weight=1.0,
                                              recon_weight=1.0, separation_weight=0.1, contrastive_weight=0.05), "32")])
def test_batched_weight_relayout_matches_per_conv(monkeypatch, cls, kw, loss, prec):
    """Steps whose dgrads read the step's one-launch weight re-layouts = steps with one re-layout launch per conv,
    bit for bit (same kernel body, same formats); the table covers the model's dgrad convs after the first step."""
    import medvae_disentangled_multimodal_amd as M
    from medvae_disentangled_multimodal_amd import ops
    dev = _dev()
    B = 16
    g = torch.Generator().manual_seed(5)
    x = (torch.randint(0, 256, (B, 3, 28, 28), generator=g).float() / 255 * 2 - 1).to(dev)
    labels = torch.zeros(B, 1, dtype=torch.long, device=dev)
    idx = torch.tensor([0, 1, 2, 3, 4, 1, 2, 4, 0, 3, 1, 2, 4, 4, 1, 2], device=dev)
    if cls == "DisentangledConditionalVAE":
        batch = (x, labels, torch.nn.functional.one_hot(idx, 12).float(), idx)
    else:
        batch = (x, labels, torch.nn.functional.one_hot(idx, 12).float())
    r = 28 // 4
    eps = [torch.randn(B, 16 if cls == "DisentangledConditionalVAE" else 8, r, r, generator=g).to(dev)
           for _ in range(3)]
    res = {}
    for batched in (False, True):
        monkeypatch.setattr(ops, "BATCHED_WT", batched)
        torch.manual_seed(11)
        model = getattr(M, cls)(**kw).to(dev)
        mod = M.VAELightningModule(model, dict(type="adam", lr=5e-4, weight_decay=0.0, betas=[0.9, 0.999]),
                                   {"type": "none"}, loss, gradient_clip_val=0.5, precision=prec)
        mod.configure_optimizers()
        losses = [mod.fit_step(batch, i, eps=eps[i]) for i in range(3)]
        torch.cuda.synchronize()
        res[batched] = (torch.stack(losses).cpu(), mod.flat.data.detach().cpu().clone())
        if batched:
            assert ops._WT.n > 0 and ops._WT.tbase == mod.flat.data.data_ptr()
    assert torch.equal(res[True][0], res[False][0])
    assert torch.equal(res[True][1], res[False][1])
